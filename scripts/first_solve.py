"""First-solve overhead of the EXACT step (table builds, allocations, graph capture) at C3
and C5: DAB_SETUP_TIMING=1 prints the phases. Usage: python scripts/first_solve.py"""
import sys, time
sys.path.insert(0, '.')
import _pkgload
pkg = _pkgload.load()
for cfg in ("c3_1kcam", "c5_rig_16x64"):
    prob = pkg.synth(**pkg.CONFIGS[cfg])
    s = pkg.Solver(0)
    t = time.perf_counter(); s.set_problem(prob.copy()); print(cfg, "set_problem %.3f s" % (time.perf_counter() - t), flush=True)
    for k in range(3):
        opts = pkg.options(max_num_iterations=1, linear_solver_type=pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR)
        t = time.perf_counter(); s.solve(opts); print(cfg, "solve(1 it) #%d %.1f ms" % (k, 1e3 * (time.perf_counter() - t)), flush=True)
    s.close()
