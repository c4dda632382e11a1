"""Summary of the persistent Cholesky's timeline (DAB_CHOL_FLOW_STAMPS=1 output on stderr,
the last factorisation in the log): per block column the diagonal tile's inputs ready, the
factor start and L_cc published (us from the kernel's start), and the bulk groups' ends.

usage: python scripts/flow_timeline.py LOG
"""
import re
import statistics as st
import sys

lines = open(sys.argv[1]).read().split("\n")
starts = [i for i, l in enumerate(lines) if l.startswith("flow n=")]
blk = lines[starts[-1]:]
cols, groups = [], []
for l in blk:
    m = re.match(r"flow col\s+(\d+)\s+(\S+)\s+(\S+)\s+(\S+)\s+\|\s+(\S+)\s+\|\s+(\S+)", l)
    if m:
        cols.append(tuple(float(x) for x in m.groups()))
    m = re.match(r"flow group\s+(\d+) bulk done\s+(\S+)", l)
    if m:
        groups.append((int(m.group(1)), float(m.group(2))))
print(f"{len(cols)} columns, total {cols[-1][3]:.1f} us")
print(f"per column (median): step {st.median([c[5] for c in cols[1:]]):.1f} us = "
      f"previous L published -> diagonal ready {st.median([cols[i][1] - cols[i - 1][3] for i in range(1, len(cols))]):.1f}"
      f" + ready -> factor start {st.median([c[2] - c[1] for c in cols]):.1f}"
      f" + factor and publish {st.median([c[4] for c in cols]):.1f}")
for q in (0, len(cols) // 4, len(cols) // 2, 3 * len(cols) // 4, len(cols) - 1):
    c = cols[q]
    print("col %3d ready %8.1f factor %8.1f published %8.1f | factor %5.1f | step %5.1f" % c)
for g, t in groups[:3] + groups[len(groups) // 2:len(groups) // 2 + 2] + groups[-2:]:
    print(f"group {g:3d} bulk done {t:8.1f}")
