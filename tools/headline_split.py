"""The headline config-2 launches' three kernels from a rocprofv3 kernel
trace of `bench.py`: python tools/headline_split.py TRACE.csv > split.json.
A launch is rows_parse -> rows_exec -> the finisher (decompress_kernel) in
dispatch order; the 1 M-block launches are the ones whose rows_exec runs
longer than 50 ms (the 65 536-block and end-to-end chunk launches are far
shorter)."""
import csv
import json
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
short = [r["Kernel_Name"].split("(")[0].replace("void ", "").replace("lz4m::", "") for r in rows]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
out = []
for i, n in enumerate(short):
    if n.startswith("rows_exec_kernel") and dur[i] > 50.0:
        p = max(j for j in range(i) if short[j].startswith("rows_parse_kernel"))
        f = next(j for j in range(i + 1, len(rows)) if short[j].startswith("decompress_kernel"))
        span = (int(rows[f]["End_Timestamp"]) - int(rows[p]["Start_Timestamp"])) / 1e6
        out.append({"parse_ms": round(dur[p], 3), "exec_ms": round(dur[i], 3), "finisher_ms": round(dur[f], 3),
                    "launch_span_ms": round(span, 3)})
avg = {k: round(sum(o[k] for o in out) / len(out), 3) for k in out[0]} if out else {}
json.dump({"source": "rocprofv3 --kernel-trace --stats -- python3 bench.py (default args)",
           "launches": out, "average": avg}, sys.stdout, indent=1)
print()
