"""Per-launch average of each PMC counter for kernels whose name contains a pattern, from
rocprofv3 --pmc csv output directories.

usage: python scripts/pmc_mix.py PATTERN DIR [DIR ...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

pat = sys.argv[1]
for d in sys.argv[2:]:
    sums, launches = defaultdict(float), defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if pat not in r["Kernel_Name"]:
                continue
            sums[r["Counter_Name"]] += float(r["Counter_Value"])
            launches[r["Counter_Name"]].add(r["Dispatch_Id"])
    print(f"{os.path.basename(d.rstrip('/'))}: kernels matching '{pat}'")
    for k in sorted(sums):
        print(f"   {k:<28} {sums[k] / max(1, len(launches[k])):14.0f}   ({len(launches[k])} launches)")
