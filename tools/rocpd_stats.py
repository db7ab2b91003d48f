"""Kernel statistics (name, calls, total/avg/min/max ns, percent) from a
rocprofv3 rocpd database: python tools/rocpd_stats.py RESULTS.db > stats.csv"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
rows = list(c.execute(
    f"select s.kernel_name, count(*), sum(d.end-d.start), avg(d.end-d.start), min(d.end-d.start), max(d.end-d.start) "
    f"from {kd} d join {ks} s on d.kernel_id = s.id group by s.kernel_name order by 3 desc"))
tot = sum(r[2] for r in rows) or 1
print('"Name","Calls","TotalDurationNs","AverageNs","MinNs","MaxNs","Percentage"')
for name, n, s, a, mn, mx in rows:
    print(f'"{name}",{n},{s},{a:.1f},{mn},{mx},{100.0 * s / tot:.3f}')
