"""Per-launch durations of k_eval_bal from a rocprofv3 --kernel-trace run, split by launch
shape: the split schedule (several ranks, or DAB_EVAL_SPLIT=1 on one) launches the kernel
twice per pass, the camera side on every CU's work-group and the point
side on the eval grid (one CU per XCD left free for the overlapped all-reduce), so the two
launches are told apart by grid size.
Usage: python scripts/split_launch_times.py <trace dir> [kernel substring]"""
import csv
import glob
import os
import statistics
import sys

d = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "k_eval_bal"
files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
if not files:
    sys.exit(f"no kernel_trace.csv under {d}")
rows = []
for f in files:
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if name in r.get("Kernel_Name", ""):
                rows.append(r)
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
by = {}
for r in rows:
    g = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
    by.setdefault(g, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
if len(by) == 1 and os.environ.get("SPLIT_ALTERNATE", "1") == "1":  # one grid: the pass's two launches alternate
    ds = next(iter(by.values()))
    by = {"camera side (1st of a pass)": ds[0::2], "point side (2nd)": ds[1::2]}
for g, ds in sorted(by.items(), key=lambda kv: str(kv[0])):
    ds_sorted = sorted(ds)
    print(f"{name} {g}: {len(ds)} launches, median {statistics.median(ds):.2f} us, "
          f"mean {statistics.mean(ds):.2f} us, p10 {ds_sorted[len(ds) // 10]:.2f} us, "
          f"p90 {ds_sorted[(9 * len(ds)) // 10]:.2f} us")
