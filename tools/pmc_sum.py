"""Sum rocprofv3 PMC csv passes for one kernel: python tools/pmc_sum.py DIR REGEX"""
import collections, csv, glob, re, sys
d, rx = sys.argv[1], sys.argv[2]
tot = collections.defaultdict(float)
n = collections.Counter()
for f in sorted(glob.glob(f"{d}/p*/p*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if re.search(rx, r.get("Kernel_Name", "")):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
for k, v in sorted(tot.items()):
    print(f"{k:32s} {v:.4g}")
if "FETCH_SIZE" in tot and "TCP_TCC_READ_REQ_sum" in tot:
    print("avg VMEM latency (cycles/instr) ~", round(tot.get("SQ_INST_LEVEL_VMEM", 0) / max(1, tot.get("SQ_INSTS_VMEM_RD", 0) + tot.get("SQ_INSTS_VMEM_WR", 0) + tot.get("SQ_INSTS_FLAT", 0)), 1))
