"""Per-step timeline of the dense Cholesky from a rocprofv3 kernel trace of chol_bench.py
(the last factorisation in the trace): panel / column update / bulk update start and end
relative to the first panel, and the gaps on the panel chain."""
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Grid_Size", "")))
rows.sort()
ch = [r for r in rows if "k_panel" in r[2] or "k_syrk" in r[2] or "k_trsv" in r[2] or "fillBuffer" in r[2]]
# last factorisation: from the last k_panel whose predecessor is a k_trsv_back (or the start)
def prev_kernel(i):  # the previous entry that is not a buffer fill (the schedule zeroes its flags first)
    j = i - 1
    while j >= 0 and "fillBuffer" in ch[j][2]:
        j -= 1
    return ch[j][2] if j >= 0 else ""
starts = [i for i, r in enumerate(ch) if "k_panel" in r[2] and (i == 0 or "k_trsv" in prev_kernel(i))]
if len(starts) < 2:  # the back substitution is not right before the next panel: split on gaps
    starts = [i for i, r in enumerate(ch) if "k_panel" in r[2] and (i == 0 or r[0] - ch[i - 1][1] > 200000)]
seg = ch[starts[-1]:]
t0 = seg[0][0]
tot = {}
for s, e, n, g in seg:
    k = n.split("(")[0].split("::")[-1]
    tot.setdefault(k, [0, 0])
    tot[k][0] += e - s
    tot[k][1] += 1
print(f"factorisation + solve: {(seg[-1][1] - t0) / 1e3:.1f} us, kernels:")
for k, (d, c) in tot.items():
    print(f"  {k:14s} n={c:4d} total {d / 1e3:9.1f} us  avg {d / c / 1e3:7.2f} us")
last_end = t0
print(" step    kernel        start      dur     gap(prev end on same kind)")
pe = {}
for i, (s, e, n, g) in enumerate(seg[:int(sys.argv[2]) if len(sys.argv) > 2 else 60]):
    k = n.split("(")[0].split("::")[-1]
    print(f" {i:4d} {k:14s} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  grid={g}")
