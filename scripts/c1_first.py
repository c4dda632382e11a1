"""Config 1's first solve on a fresh handle, phase by phase (set-up, solve), three fresh
handles in a row; with DAB_SETUP_TIMING=1 the library prints its phase times on stderr."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
prob = pkg.synth(**pkg.CONFIGS["c1_rig_8x36"])
o1 = pkg.options(max_num_iterations=10)
for r in range(3):
    p = prob.copy()
    t0 = time.perf_counter()
    s = pkg.Solver(0)
    t1 = time.perf_counter()
    s.set_problem(p)
    t2 = time.perf_counter()
    summ = s.solve(o1)
    t3 = time.perf_counter()
    s.close()
    t4 = time.perf_counter()
    its = [1e3 * it["time"] for it in summ["iterations"]]
    print(f"rep {r}: create {1e3*(t1-t0):.2f} ms  set_problem {1e3*(t2-t1):.2f} ms  solve {1e3*(t3-t2):.2f} ms "
          f"(iterations {' '.join(f'{x:.2f}' for x in its)})  destroy {1e3*(t4-t3):.2f} ms", flush=True)
