"""BASELINE config 5 rig (16 x 64, 1M points, 10M observations), the exact step
(DENSE_SCHUR: block tiles + dense Cholesky) for a few LM iterations: the driver of the
k_schur_y / k_schur_tiles profiles. usage: python scripts/rig_explicit.py [iterations] [config]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import _pkgload  # noqa: E402

pkg = _pkgload.load()
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
cfg = sys.argv[2] if len(sys.argv) > 2 else "c5_rig_16x64"
prob = pkg.synth(**pkg.CONFIGS[cfg])
s = pkg.Solver(0)
t0 = time.perf_counter()
s.set_problem(prob)
print(f"{cfg}: set_problem {time.perf_counter() - t0:.3f} s", flush=True)
summ = s.solve(pkg.options(max_num_iterations=iters, linear_solver_type=pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR,
                           function_tolerance=0.0, parameter_tolerance=0.0, gradient_tolerance=0.0))
its = [it["time"] for it in summ["iterations"][1:]]
print(f"explicit: {summ['num_iterations']} iterations, median {1e3 * np.median(its):.2f} ms/iter, "
      f"costs {[it['cost'] for it in summ['iterations']]}", flush=True)
s.close()
