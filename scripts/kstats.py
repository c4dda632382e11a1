"""Per-kernel summary of a rocprofv3 SQLite output: python scripts/kstats.py <dir-or-db> [top]"""
import glob
import os
import sqlite3
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
db = path if path.endswith(".db") else glob.glob(os.path.join(path, "*.db"))[0]
c = sqlite3.connect(db)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
q = (f"select s.kernel_name, count(*), avg(d.end-d.start)/1000.0, sum(d.end-d.start)/1e6, "
     f"min(d.end-d.start)/1000.0 from {kd} d join {ks} s on d.kernel_id=s.id group by s.kernel_name "
     f"order by 4 desc limit {top}")
print(f"{'total_ms':>9} {'calls':>6} {'avg_us':>10} {'min_us':>10}  kernel")
for name, n, avg, tot, mn in c.execute(q):
    print(f"{tot:9.3f} {n:6d} {avg:10.2f} {mn:10.2f}  {name[:120]}")
