"""Counter calibration report (tools/pmc_cal.sh): for each known-bytes kernel
of tools/micro/traffic_cal, the byte estimates of every counting method
divided by the bytes the kernel moves (1.00 = exact).

Methods (per dispatch):
  fetch2      2 x FETCH_SIZE (the MI355X guide: FETCH_SIZE tallies 128-B
              requests at 64 B)
  rdreq_sized 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B (+ 64 B for the
              requests of no listed size)
  rdreq128    128 * TCC_EA0_RDREQ
  write_size  WRITE_SIZE
  wrreq_sized 64*WRREQ_64B + 32*(WRREQ - WRREQ_64B)
  wrreq64     64 * TCC_EA0_WRREQ
"""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
known = {}
for line in open(f"{d}/plain.log"):
    line = line.strip()
    if line.startswith("{"):
        r = json.loads(line)
        known[r["kernel"]] = r
ctr = collections.defaultdict(dict)
for f in sorted(glob.glob(f"{d}/p*/p*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = next((n for n in known if r["Kernel_Name"].startswith(n) or f" {n}(" in r["Kernel_Name"]
                  or r["Kernel_Name"].split("(")[0].endswith(n)), None)
        if k is None:
            continue
        ctr[k][r["Counter_Name"]] = ctr[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])


def methods(c):
    rd_other = c.get("TCC_EA0_RDREQ_sum", 0) - c.get("TCC_EA0_RDREQ_32B_sum", 0) - c.get("TCC_EA0_RDREQ_64B_sum", 0) \
        - c.get("TCC_EA0_RDREQ_128B_sum", 0)
    return {
        "fetch2": 2 * 1024 * c.get("FETCH_SIZE", 0),
        "rdreq_sized": 32 * c.get("TCC_EA0_RDREQ_32B_sum", 0) + 64 * c.get("TCC_EA0_RDREQ_64B_sum", 0)
        + 128 * c.get("TCC_EA0_RDREQ_128B_sum", 0) + 64 * max(rd_other, 0),
        "rdreq128": 128 * c.get("TCC_EA0_RDREQ_sum", 0),
        "write_size": 1024 * c.get("WRITE_SIZE", 0),
        "wrreq_sized": 64 * c.get("TCC_EA0_WRREQ_64B_sum", 0)
        + 32 * (c.get("TCC_EA0_WRREQ_sum", 0) - c.get("TCC_EA0_WRREQ_64B_sum", 0)),
        "wrreq64": 64 * c.get("TCC_EA0_WRREQ_sum", 0),
    }


out = {}
for k, kn in known.items():
    c = ctr.get(k, {})
    m = methods(c)
    row = {"known_read": kn["read"], "known_write": kn["write"], "ms": kn["ms"], "counters": c}
    for name, v in m.items():
        ref = kn["read"] if name in ("fetch2", "rdreq_sized", "rdreq128") else kn["write"]
        row[name] = v
        row[name + "_ratio"] = round(v / ref, 4) if ref else None
    out[k] = row
print(json.dumps(out, indent=1))
