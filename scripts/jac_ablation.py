"""Interleaved in-process A/B of residual+Jacobian kernel variants (HIP-event kernel time).

Variants (DAB_JAC_VARIANT): low bits = parts skipped (1 records, 2 V/g scan, 4 Jp planes),
hundreds = __launch_bounds__ waves/SIMD (0 -> 2, 100 -> 3, 200 -> 4). Prints median/min ms.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3_1kcam"
variants = [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else
                             "0,100,200,1,2,3,7,201,203,207".split(","))]
prob = pkg.synth(**pkg.CONFIGS[cfg])
s = pkg.Solver(0)
s.set_problem(prob)
res = {v: [] for v in variants}
for rnd in range(8):
    for v in variants:
        os.environ["DAB_JAC_VARIANT"] = str(v)
        for _ in range(3):
            s.bench_eval_pass(False)
        s.bench_kernel_ms()
        for _ in range(10):
            s.bench_eval_pass(False)
        res[v].append(s.bench_kernel_ms()[0])
os.environ.pop("DAB_JAC_VARIANT")
nbytes = s.jacobian_bytes()
for v in variants:
    a = np.array(res[v])
    print(f"variant {v:4d}: median {np.median(a)*1e3:8.2f} us  min {a.min()*1e3:8.2f} us  "
          f"alg GB/s {nbytes/np.median(a)/1e6:8.1f}")
s.close()
