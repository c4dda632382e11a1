"""C3 (1000 cameras, 1M observations) implicit-Schur PCG only, fp64 or fp32 Schur factors:
one warm-up solve, then `iters` LM iterations; for a kernel-trace breakdown.
Usage: python scripts/c3_pcg_only.py [iters] [fp32]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
f32 = int(sys.argv[2]) if len(sys.argv) > 2 else 0
prob = pkg.synth(**pkg.CONFIGS["c3_1kcam"])
s = pkg.Solver(0)
s.set_problem(prob)
pts0, ext0 = prob.points.copy(), prob.ext.copy()
opts = pkg.options(max_num_iterations=iters, function_tolerance=0.0, gradient_tolerance=0.0,
                   parameter_tolerance=0.0, pcg_fp32=f32, linear_solver_type=pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)
for rep in range(2):
    s.update_parameters(pts0, ext0)
    t = time.perf_counter()
    r = s.solve(opts)
    its = [it["time"] * 1e3 for it in r["iterations"][1:]]
    print(f"rep {rep}: wall {1e3 * (time.perf_counter() - t):.1f} ms, iter ms {[round(x, 3) for x in its]}, "
          f"cg {[it['linear_solver_iterations'] for it in r['iterations'][1:]]}", flush=True)
s.close()
