"""Kernel timeline of LM iterations (run under rocprofv3 --kernel-trace): config, linear
solver and fp32 flag from the command line. Prints nothing itself but the summary; the
trace CSV is analysed afterwards (scripts/timeline.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import _pkgload  # noqa: E402

pkg = _pkgload.load()
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3_1kcam"
lst = int(sys.argv[2]) if len(sys.argv) > 2 else pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG
f32 = int(sys.argv[3]) if len(sys.argv) > 3 else 0
prob = pkg.synth(**pkg.CONFIGS[cfg])
s = pkg.Solver(0)
s.set_problem(prob)
summ = s.solve(pkg.options(max_num_iterations=6, linear_solver_type=lst, function_tolerance=0.0, pcg_fp32=f32,
                           parameter_tolerance=0.0, gradient_tolerance=0.0))
its = [it["time"] for it in summ["iterations"][1:]]
print(f"{cfg} solver {lst} fp32={f32}: median {1e3 * np.median(its):.3f} ms/iter, "
      f"cg {[it['linear_solver_iterations'] for it in summ['iterations'][1:]]}", flush=True)
s.close()
