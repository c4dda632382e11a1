import sys, time
sys.path.insert(0, '.')
import _pkgload
pkg = _pkgload.load()
for cfg in ("c5_rig_16x64", "c3_1kcam"):
    prob = pkg.synth(**pkg.CONFIGS[cfg])
    s = pkg.Solver(0)
    for k in range(2):
        t = time.perf_counter(); s.set_problem(prob); print(cfg, "set_problem %.3f s" % (time.perf_counter() - t), flush=True)
    s.close()
