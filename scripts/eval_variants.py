"""Point-kernel variant sweep: eval-pass timing per DAB_EVAL_WPS value, plus a short PCG
solve whose trajectory must match the first variant's (bitwise for the same row split).

usage: python scripts/eval_variants.py CONFIG WPS [WPS ...]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
cfg = sys.argv[1]
variants = sys.argv[2:]  # DAB_EVAL_WPS values (two-kernel pass), "fused[SIDE]", "tab" or "split"
base = pkg.synth(**pkg.CONFIGS[cfg])
ref = None
for wps in variants:
    for k in ("DAB_EVAL_SPLIT", "DAB_EVAL_SIDE", "DAB_FUSED_TAB", "DAB_EVAL_WPS"):
        os.environ.pop(k, None)
    if wps == "split":  # the multi-rank schedule (camera-side, then point-side launch)
        os.environ["DAB_EVAL_FUSED"] = "1"
        os.environ["DAB_EVAL_SPLIT"] = "1"
    elif wps.startswith("fused"):  # k_eval_bal; fused<N>: DAB_EVAL_SIDE=N timing ablation
        os.environ["DAB_EVAL_FUSED"] = "1"
        os.environ["DAB_FUSED_TAB"] = "0"
        os.environ["DAB_EVAL_SIDE"] = wps[5:] or "0"
    elif wps == "tab":  # k_eval_bal reading the tables of the current x
        os.environ["DAB_EVAL_FUSED"] = "1"
        os.environ["DAB_FUSED_TAB"] = "1"
    else:
        os.environ["DAB_EVAL_FUSED"] = "0"
        os.environ["DAB_EVAL_WPS"] = str(wps)
    os.environ["DAB_BENCH_SAMPLE"] = "8"
    prob = base.copy()
    s = pkg.Solver(0)
    s.set_problem(prob)
    s.bench_eval_pass(True, 5)
    s.sync()
    s.bench_kernel_ms()
    t0 = time.perf_counter()
    s.bench_eval_pass(True, 50)
    s.sync()
    dt = (time.perf_counter() - t0) / 50
    j, a = s.bench_kernel_ms()
    g = s.solve(pkg.options(max_num_iterations=3, linear_solver_type=pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG))
    s.close()
    costs = [it["cost"] for it in g["iterations"]]
    if ref is None:
        ref = (costs, prob.points.copy())
        diff = "reference"
    else:
        dc = max(abs(x - y) / max(abs(y), 1e-300) for x, y in zip(costs, ref[0])) if len(costs) == len(ref[0]) else float("nan")
        dx = float(np.abs(prob.points - ref[1]).max())
        diff = f"cost rel diff {dc:.2e}, max |dX| {dx:.2e}"
    print(f"{cfg} wps={wps}: step {dt * 1e3:.4f} ms, points kernel {j * 1e3:.1f} us, rest {a * 1e3:.1f} us, "
          f"{prob.num_obs / dt / 1e6:.0f} M obs/s | {diff}", flush=True)
