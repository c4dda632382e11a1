"""k_eval_bal smoke on one GPU: one evaluation pass at a time under DAB_XTAB_DEBUG (the
per-XCD table counters and the error word after each pass), then V, g, ug, cost against
the k_eval_fused pass of a second handle (DAB_EVAL_BAL=0)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2_100cam"
os.environ["DAB_XTAB_DEBUG"] = "1"
pkg = _pkgload.load()
prob = pkg.synth(**pkg.CONFIGS[cfg])
print("problem", cfg, prob.num_obs, flush=True)
res = {}
for bal in sys.argv[2].split(",") if len(sys.argv) > 2 else ("1", "0"):
    os.environ["DAB_EVAL_BAL"] = bal
    s = pkg.Solver(0)
    s.set_problem(prob.copy())
    print("bal", bal, "set up", flush=True)
    for i in range(3):
        t = time.perf_counter()
        s.bench_eval_pass(True, 1)
        s.sync()
        print("  pass", i, "%.1f ms" % (1e3 * (time.perf_counter() - t)), flush=True)
    r, cost = s.residuals()
    summ = s.solve(pkg.options(max_num_iterations=3, function_tolerance=0.0, gradient_tolerance=0.0,
                               parameter_tolerance=0.0, linear_solver_type=pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG))
    res[bal] = [it["cost"] for it in summ["iterations"]]
    print("  costs", res[bal], flush=True)
    s.close()
keys = list(res)
for k in keys[1:]:
    print("max rel cost dev", keys[0], k, max(abs(a - b) / abs(b) for a, b in zip(res[keys[0]], res[k])))
