"""Per-launch counters of the decoder dispatches in a tools/pmc_bench.sh run.

One decoder launch = the row decoder's three kernels (parse, execution,
finisher); the k-th dispatch of each kernel belongs to launch k.  Launch
order in `bench.py --steps 1 --warmup 0 --no-compress`: launch 0 is the
silesia-like headline launch (config 2), then the 65 536-block mid-batch
launches, and the LAST launch is a random-data launch, whose bytes are known
(pure streaming: read ~= compressed size, write = decoded size) and serves as
a check of the method on the decoder itself.  The summary carries the hash of the decoder sources
(bench.decoder_src_sha) so bench.py reports roofline.traffic only for the
kernels that were profiled."""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = tuple(os.environ.get("PMC_KERNELS", "rows_parse_kernel,rows_exec_kernel,decompress_kernel<false, true>").split(","))
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

# ---- HBM bytes per launch, the MI355X guide's method (MI355X_MICROARCH.md,
# HBM section): separate --pmc passes; read = 2 x FETCH_SIZE (gfx950 tallies
# 128-B requests at 64 B), write = WRITE_SIZE (exact for 16-B-per-lane
# stores).  The request-size breakdown (RDREQ_32B/64B/128B, WRREQ_64B) is kept
# for reference only: its write estimate read 0.75x the known bytes of a
# streaming dispatch.  tools/pmc_cal.sh checks both methods on kernels of
# known bytes in the decoder's access shapes (profiles/r03/*calibration*).
def hbm_bytes(c):
    return 2 * 1024 * c.get("FETCH_SIZE", 0), 1024 * c.get("WRITE_SIZE", 0)


def hbm_bytes_reqsize(c):
    rd = 32 * c.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * c.get("TCC_EA0_RDREQ_64B_sum", 0) \
        + 128 * c.get("TCC_EA0_RDREQ_128B_sum", 0)
    wr = 64 * c.get("TCC_EA0_WRREQ_64B_sum", 0) + 32 * (c.get("TCC_EA0_WRREQ_sum", 0) - c.get("TCC_EA0_WRREQ_64B_sum", 0))
    return rd, wr


sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 2:
    head, rand = out[0], (out[max(out)] if len(out) > 1 else None)
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
        "method": "read = 2 x FETCH_SIZE, write = WRITE_SIZE (MI355X guide, HBM section; one counter group per "
                  "rocprofv3 --pmc pass); calibrated on known-bytes kernels by tools/pmc_cal.sh",
        "reqsize_method_read_bytes": hbm_bytes_reqsize(head)[0],
        "reqsize_method_write_bytes": hbm_bytes_reqsize(head)[1],
    }
    cal = sys.argv[5] if len(sys.argv) > 5 else None
    if cal and os.path.exists(cal):
        summary["calibration"] = {k: {m: v.get(m + "_ratio") for m in ("fetch2", "rdreq_sized", "write_size",
                                                                        "wrreq_sized")}
                                  for k, v in json.load(open(cal)).items()}
    if rand:
        rrd, rwr = hbm_bytes(rand)
        summary["random_dispatch"] = {"read_bytes": rrd, "write_bytes": rwr,
                                      "note": "131072 random (stored-like) blocks: the finisher's lane-per-block "
                                              "literal copies; write = 131072 * 65536 = 8.59e9 bytes must leave, "
                                              "reads ~= 8.62e9 compressed bytes plus any line re-fetches"}
    with open(sys.argv[2], "w") as f:
        json.dump(summary, f, indent=1)
