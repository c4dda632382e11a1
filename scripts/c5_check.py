"""BASELINE config 5 (rig 16 x 64, 1M points, 10M observations) on one GPU: set-up time,
evaluation-pass throughput and LM iterations with the PCG step."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import _pkgload  # noqa: E402

pkg = _pkgload.load()
cfg = sys.argv[1] if len(sys.argv) > 1 else "c5_rig_16x64"
t0 = time.perf_counter()
prob = pkg.synth(**pkg.CONFIGS[cfg])
t1 = time.perf_counter()
pts0, ext0 = prob.points.copy(), prob.ext.copy()
s = pkg.Solver(0)
s.set_problem(prob)
t2 = time.perf_counter()
print(f"{cfg}: {prob.num_obs} obs, synth {t1 - t0:.1f} s, set_problem {t2 - t1:.1f} s", flush=True)
s.bench_eval_pass(True, 3)
s.sync()
s.bench_kernel_ms()
t3 = time.perf_counter()
s.bench_eval_pass(True, 10)
s.sync()
dt = (time.perf_counter() - t3) / 10
j, a = s.bench_kernel_ms()
print(f"eval pass {dt * 1e3:.3f} ms ({prob.num_obs / dt / 1e6:.0f} M obs/s), point kernel {j:.3f} ms, "
      f"camera side {a:.3f} ms", flush=True)
for lst, f32 in ((pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG, 0), (pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG, 1),
                 (pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR, 0)):
    try:
        summ = s.solve(pkg.options(max_num_iterations=4, linear_solver_type=lst, function_tolerance=0.0, pcg_fp32=f32,
                                   parameter_tolerance=0.0, gradient_tolerance=0.0))
        its = [it["time"] for it in summ["iterations"][1:]]
        print(f"solver {lst} fp32={f32}: {summ['num_iterations']} iterations, median {1e3 * np.median(its):.2f} ms/iter, "
              f"cost {summ['initial_cost']:.6e} -> {summ['final_cost']:.6e}, "
              f"cg {[it['linear_solver_iterations'] for it in summ['iterations'][1:]]}", flush=True)
    except RuntimeError as e:
        print(f"solver {lst}: {e}", flush=True)
    s.update_parameters(pts0, ext0)
s.close()
