"""Summarise rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE, collected in separate runs)
into per-kernel HBM bytes per launch, and write the k_jacobian figure that bench.py
reports as roofline.traffic.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half of the
bytes of wide coalesced streaming reads, so it is doubled; WRITE_SIZE is taken as is.
Both counters are in KiB. Usage:
  python scripts/traffic.py FETCH_DIR WRITE_DIR OUT_JSON --config c3_1kcam --n-obs 1000000
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(d, counter):
    per = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                per[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return per


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("dab::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("out")
    ap.add_argument("--config", default="c3_1kcam")
    ap.add_argument("--n-obs", type=int, default=1000000)
    ap.add_argument("--valu-dir", default="", help="a third PMC pass with SQ_INSTS_VALU (wave-instructions)")
    ap.add_argument("--lib", default="", help="the libdab.so profiled (its sha256 goes into the record; "
                    "bench.py reports the traffic only for that exact binary)")
    ap.add_argument("--kernel", default="auto", help="kernel name prefix (auto: k_eval_bal if it ran, "
                    "else k_eval_points)")
    a = ap.parse_args()
    fetch, write = load(a.fetch_dir, "FETCH_SIZE"), load(a.write_dir, "WRITE_SIZE")
    valu = load(a.valu_dir, "SQ_INSTS_VALU") if a.valu_dir else {}
    table = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fb = 2.0 * 1024 * sum(f) / len(f) if f else None
        wb = 1024.0 * sum(w) / len(w) if w else None
        v = valu.get(k, [])
        table[short(k)] = dict(launches=max(len(f), len(w)), fetch_bytes_x2=fb, write_bytes=wb,
                               bytes_per_launch=(fb or 0.0) + (wb or 0.0),
                               valu_insts=(sum(v) / len(v)) if v else None)
    if a.kernel == "auto":
        a.kernel = "k_eval_bal" if any(k.startswith("k_eval_bal") for k in table) else "k_eval_points"
    # the evaluation-kernel variant the bench ran (most launches among the matching names)
    main_k = sorted((k for k in table if k.startswith(a.kernel)), key=lambda k: -table[k]["launches"])
    lib_sha = None
    if a.lib:
        import hashlib
        lib_sha = hashlib.sha256(open(a.lib, "rb").read()).hexdigest()
    out = dict(config=a.config, n_obs=a.n_obs, kernel=main_k[0] if main_k else None, libdab_sha256=lib_sha,
               bytes_per_launch=table[main_k[0]]["bytes_per_launch"] if main_k else None,
               valu_insts_per_launch=table[main_k[0]]["valu_insts"] if main_k else None,
               correction="FETCH_SIZE x2 (gfx950 wide-load tally), WRITE_SIZE x1, KiB->B",
               kernels=table)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, v in sorted(table.items(), key=lambda kv: -kv[1]["bytes_per_launch"]):
        print(f"{k:60s} {v['launches']:5d} {v['bytes_per_launch'] / 1e6:10.2f} MB/launch")


if __name__ == "__main__":
    main()
