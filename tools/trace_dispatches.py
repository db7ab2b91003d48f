"""Per-dispatch durations (ms) of the bench's kernels from a rocprofv3
kernel_trace.csv: python tools/trace_dispatches.py TRACE.csv > dispatches.json.
The headline decoder launches are the bench's timed config-2 dispatches
(the ones with the modal grid over 1 M blocks); the rest are listed apart."""
import collections
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"]
    ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    by[name].append(round(ms, 3))
out = {"source": "rocprofv3 --kernel-trace --stats -- python3 bench.py (default args)"}
for name, ds in by.items():
    short = name.split("(")[0].replace("void ", "").replace("lz4m::", "")
    if not any(k in short for k in ("decompress", "compress", "xxh32")):
        continue
    ent = {"dispatches_ms": ds, "avg_ms": round(sum(ds) / len(ds), 3)}
    if short.startswith("stage_decompress_kernel"):
        # the 1 M-block config-2 launches: the compress check's decode, the
        # warmup and the timed steps (the e2e chunks, random blocks and the
        # 4 MiB-block frame decode are far shorter or longer)
        big = [d for d in ds if 150.0 < d < 1000.0]
        ent["headline_dispatches_ms"] = big
        ent["headline_avg_ms"] = round(sum(big) / max(1, len(big)), 3)
    out[short] = ent
json.dump(out, sys.stdout, indent=1)
