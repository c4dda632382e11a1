"""Prints the exact LM cost trajectory of a few solves (rig PCG fp64 / mixed, rig exact,
BAL PCG) for A/B checks of kernel variants selected by environment knobs: two runs with
different knobs must print the same lines when the variants are bitwise equivalent.
Usage: python scripts/ab_costs.py [config]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
cfg = sys.argv[1] if len(sys.argv) > 1 else "c5_rig_16x64"
prob = pkg.synth(**pkg.CONFIGS[cfg])
s = pkg.Solver(0)
s.set_problem(prob)
pts0, ext0 = prob.points.copy(), prob.ext.copy()
for name, lst, f32 in (("pcg64", pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG, 0),
                       ("pcg32", pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG, 1),
                       ("exact", pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR, 0)):
    s.update_parameters(pts0, ext0)
    r = s.solve(pkg.options(max_num_iterations=4, pcg_fp32=f32, linear_solver_type=lst))
    print(name, [it["cost"].hex() for it in r["iterations"]],
          [it["linear_solver_iterations"] for it in r["iterations"]], flush=True)
s.close()
