"""C5 rig (16 x 64, 1M points, 10M observations): LM iterations with the exact dense-Schur
step (DENSE_SCHUR; S from the fixed-point tiles) and with the matrix-free PCG, per-iteration
wall-clock. Usage: python scripts/rig_explicit.py [iters] [config]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
cfg = sys.argv[2] if len(sys.argv) > 2 else "c5_rig_16x64"
t = time.perf_counter()
prob = pkg.synth(**pkg.CONFIGS[cfg])
print(f"synth {time.perf_counter() - t:.2f} s, {prob.num_obs} obs", flush=True)
s = pkg.Solver(0)
t = time.perf_counter()
s.set_problem(prob)
print(f"set_problem {time.perf_counter() - t:.2f} s", flush=True)
pts0, ext0 = prob.points.copy(), prob.ext.copy()
for name, lst in (("explicit", pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR), ("pcg", pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG),
                  ("explicit", pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR)):
    s.update_parameters(pts0, ext0)
    t = time.perf_counter()
    r = s.solve(pkg.options(max_num_iterations=iters, function_tolerance=0.0, gradient_tolerance=0.0,
                            parameter_tolerance=0.0, linear_solver_type=lst))
    wall = time.perf_counter() - t
    its = [it["time"] * 1e3 for it in r["iterations"][1:]]
    print(f"{name}: wall {wall * 1e3:.1f} ms, iter ms {np.round(its, 3).tolist()}, median {np.median(its):.3f}, "
          f"linear {r['linear_solver_time'] * 1e3:.1f} ms, assembly {r['schur_assembly']}, "
          f"costs {['%.10e' % it['cost'] for it in r['iterations']]}", flush=True)
s.close()
