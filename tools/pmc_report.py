"""Per-launch counters of the decoder dispatches in a tools/pmc_bench.sh run.

One decoder launch = the row decoder's three kernels (parse, execution,
finisher); the k-th dispatch of each kernel belongs to launch k.  Launch
order in `bench.py --steps 1 --warmup 0 --no-compress`: launch 0 is the
silesia-like headline launch (config 2); the next two are the random-data
launches (warmup + step), whose bytes are known (pure streaming: read ~=
compressed size, write = decoded size) and serve as the calibration of the
request counters.  The summary carries the hash of the decoder sources
(bench.decoder_src_sha) so bench.py reports roofline.traffic only for the
kernels that were profiled."""
import collections
import csv
import glob
import json
import sys

import os

KERNELS = ("rows_parse_kernel", "rows_exec_kernel", "decompress_kernel<false, true>")
d = sys.argv[1]
per = collections.defaultdict(dict)   # launch order -> counter -> value
for f in sorted(glob.glob(f"{d}/p*/p*_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    for kn in KERNELS:
        kr = [r for r in rows if kn in r["Kernel_Name"]]
        order = sorted({int(r["Dispatch_Id"]) for r in kr})
        for r in kr:
            k = order.index(int(r["Dispatch_Id"]))
            per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
out = {k: v for k, v in sorted(per.items())}
print(json.dumps(out, indent=1))

# ---- HBM bytes per launch (guide: separate passes; request-size counters,
# calibrated here on the random-data dispatch whose bytes are known) ----
def hbm_bytes(c):
    rd = 32 * c.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * c.get("TCC_EA0_RDREQ_64B_sum", 0) \
        + 128 * c.get("TCC_EA0_RDREQ_128B_sum", 0)
    wr = 64 * c.get("TCC_EA0_WRREQ_64B_sum", 0) + 32 * (c.get("TCC_EA0_WRREQ_sum", 0) - c.get("TCC_EA0_WRREQ_64B_sum", 0))
    return rd, wr


sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 2:
    head, rand = out[0], out.get(1)
    rd, wr = hbm_bytes(head)
    summary = {
        "kernel": "+".join(KERNELS),
        "decoder_src_sha": __import__("importlib").import_module("bench").decoder_src_sha(),
        "command": "bench.py (config 2 workload) under rocprofv3 --pmc, one counter group per pass (tools/pmc_bench.sh)",
        "blocks": int(sys.argv[3]) if len(sys.argv) > 3 else 1048576,
        "pool": int(sys.argv[4]) if len(sys.argv) > 4 else 4096,
        "hbm_read_bytes_per_launch": rd,
        "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr,
        "fetch_size_kb": head.get("FETCH_SIZE"),
        "write_size_kb": head.get("WRITE_SIZE"),
        "l2_hit": head.get("TCC_HIT_sum"),
        "method": "read = 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B, write = 64*WRREQ_64B + 32*(WRREQ - WRREQ_64B); "
                  "FETCH_SIZE reads exactly half of this (MI355X guide: 128-B requests tallied at 64 B)",
    }
    if rand:
        rrd, rwr = hbm_bytes(rand)
        summary["calibration_random_dispatch"] = {"read_bytes": rrd, "write_bytes": rwr,
                                                 "note": "131072 random blocks: expected read ~= compressed bytes "
                                                         "(~8.62e9), write = 131072 * 65536 = 8.59e9"}
    with open(sys.argv[2], "w") as f:
        json.dump(summary, f, indent=1)
