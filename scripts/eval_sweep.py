"""Tuning sweep of the evaluation pass (camera chunk size) on one config."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3_1kcam"
prob = pkg.synth(**pkg.CONFIGS[cfg])
for wps, chunk, noev in ((-2, 4096, 0), (-5, 4096, 0), (42, 4096, 0), (41, 4096, 0)):
    os.environ["DAB_CHUNK"] = str(chunk)
    os.environ["DAB_EVAL_WPS"] = str(wps)
    os.environ["DAB_BENCH_SAMPLE"] = "0" if noev else "8"
    s = pkg.Solver(0)
    s.set_problem(prob)
    s.bench_eval_pass(True, 5)
    s.sync()
    s.bench_kernel_ms()
    t0 = time.perf_counter()
    s.bench_eval_pass(True, 30)
    s.sync()
    dt = (time.perf_counter() - t0) / 30
    j, a = s.bench_kernel_ms() if not noev else (0.0, 0.0)
    print(f"{cfg} wps={wps} chunk={chunk} noev={noev}: step {dt * 1e3:.3f} ms, points kernel {j * 1e3:.1f} us, rest {a * 1e3:.1f} us, "
          f"{prob.num_obs / dt / 1e6:.0f} M obs/s", flush=True)
    s.close()
