"""Dispatch-ordered durations (ms) of the row decoder's kernels from a
rocprofv3 kernel_trace.csv: python tools/dispatch_seq.py TRACE.csv
(one line per dispatch of rows_parse / rows_exec / the finisher)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    name = r["Kernel_Name"]
    short = name.split("(")[0].replace("void ", "").replace("lz4m::", "")
    if not any(k in short for k in ("rows_parse", "rows_exec", "decompress_kernel")):
        continue
    ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    print(f"{short[:40]:40s} {ms:9.3f}")
