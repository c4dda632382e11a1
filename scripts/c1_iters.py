"""Config-1 rig (8 x 36, 20k points): per-iteration wall-clock of a solve on a fresh handle,
after a re-set of the same problem on that handle (the sfm.cc loop's pattern), and a warm
re-solve. usage: python scripts/c1_iters.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
prob = pkg.synth(**pkg.CONFIGS["c1_rig_8x36"])
p0, e0 = prob.points.copy(), prob.ext.copy()
o = pkg.options(max_num_iterations=10)
t = time.perf_counter()
s = pkg.Solver(0)
print(f"handle creation {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
for tag in ("cold", "reset", "warm"):
    t = time.perf_counter()
    if tag != "warm":
        prob.points[:], prob.ext[:] = p0, e0
        s.set_problem(prob)
    else:
        s.update_parameters(p0, e0)
    s.sync()
    if os.environ.get("C1_SLEEP"):
        time.sleep(float(os.environ["C1_SLEEP"]))
    ts = time.perf_counter()
    g = s.solve(o)
    te = time.perf_counter()
    print(f"{tag}: set {1e3 * (ts - t):.2f} ms, solve {1e3 * (te - ts):.2f} ms, iterations (ms) "
          f"{[round(1e3 * it['time'], 3) for it in g['iterations']]}", flush=True)
s.close()
