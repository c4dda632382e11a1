"""Summarise a rocprofv3 kernel trace between two launches of a marker kernel: busy time,
per-kernel totals, and idle gaps (host waits, launch latency)."""
import csv
import sys
from collections import defaultdict

path, marker = sys.argv[1], sys.argv[2]
which = int(sys.argv[3]) if len(sys.argv) > 3 else 2
rows = list(csv.DictReader(open(path)))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dab::", "")) for r in rows)
idx = [i for i, k in enumerate(ks) if k[2].startswith(marker)]
a, b = idx[which], idx[which + 1]
seg = ks[a:b]
span = ks[b][0] - seg[0][0]
busy = sum(e - s for s, e, _ in seg)
print(f"span {span / 1e3:.1f} us, kernel busy {busy / 1e3:.1f} us, {len(seg)} kernels")
agg = defaultdict(lambda: [0, 0])
for s, e, n in seg:
    agg[n][0] += 1
    agg[n][1] += e - s
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:20]:
    print(f"  {n[:40]:40s} {c:4d} {t / 1e3:9.1f} us")
prev, gaps = seg[0][1], []
for s, e, n in seg[1:]:
    if s - prev > 3000:
        gaps.append(((s - prev) / 1e3, n))
    prev = max(prev, e)
print(f"gaps > 3 us: {len(gaps)}, total {sum(g for g, _ in gaps):.1f} us")
for g, n in sorted(gaps, reverse=True)[:12]:
    print(f"   {g:7.1f} us before {n}")
