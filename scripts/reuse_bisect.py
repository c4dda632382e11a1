"""Which earlier solve on the same handle changes a later large-camera PCG trajectory?
Prints the LM costs of the large rig PCG solve after each prefix of solves."""
import sys
sys.path.insert(0, '.')
import _pkgload
pkg = _pkgload.load()
small = pkg.synth(kind=1, num_arcs=4, num_rings=10, num_points=1500, obs_per_point=6, seed=81)
large = pkg.synth(kind=1, num_arcs=12, num_rings=160, num_points=6000, obs_per_point=8, seed=82)
PCG, EXP = pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG, pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR


def run(s, prob, lst):
    p = prob.copy()
    s.set_problem(p)
    r = s.solve(pkg.options(max_num_iterations=4, linear_solver_type=lst))
    return [it["cost"] for it in r["iterations"]], [it["linear_solver_iterations"] for it in r["iterations"]]


for name, prefix in (("fresh", []), ("large twice", [(large, PCG)]), ("small pcg", [(small, PCG)]),
                     ("small explicit", [(small, EXP)]), ("small pcg+explicit", [(small, PCG), (small, EXP)])):
    s = pkg.Solver(0)
    for prob, lst in prefix:
        run(s, prob, lst)
    c, it = run(s, large, PCG)
    s.close()
    print(f"{name:22s} {[repr(x) for x in c]} {it}", flush=True)
