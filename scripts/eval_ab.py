"""A/B timing of evaluation-pass variants on one GPU (knobs are read when a handle is
created, so each variant gets its own handle with its environment set first).

usage: python scripts/eval_ab.py CONFIG REPS NAME=ENV1=V1,ENV2=V2 [NAME=...]
  (a bare NAME with no '=' runs the defaults; LIB=path runs that build of libdab instead)

Per variant and rep: step wall time over 200 back-to-back passes, the kernel's HIP-event
mean, and a 3-iteration PCG LM solve whose per-iteration costs are compared with the first
variant's (relative difference printed; the variants must agree to rounding).
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

KNOBS = ("DAB_EVAL_FUSED", "DAB_FUSED_TAB", "DAB_EVAL_SIDE", "DAB_EVAL_SPLIT")


DEFAULT_LIB = []


def parse(spec):
    name, _, rest = spec.partition("=")
    env = {}
    for kv in filter(None, rest.split(",")):
        k, _, v = kv.partition("=")
        env[k] = v
    return name, env


def run(pkg, prob, env, passes=200):
    abi = sys.modules[pkg.__name__ + "._abi"]
    env = dict(env)
    lib = env.pop("LIB", None)
    abi._LIB = abi.load_library(os.path.join(ROOT, lib)) if lib else DEFAULT_LIB[0]
    for k in KNOBS:
        os.environ.pop(k, None)
    os.environ.update(env)
    s = pkg.Solver(0)
    s.set_problem(prob.copy())
    s.bench_eval_pass(True, 20)
    s.sync()
    s.bench_kernel_ms()
    t = time.perf_counter()
    s.bench_eval_pass(True, passes)
    s.sync()
    step = (time.perf_counter() - t) / passes
    kern, _ = s.bench_kernel_ms()
    summ = s.solve(pkg.options(max_num_iterations=3, function_tolerance=0.0, gradient_tolerance=0.0,
                               parameter_tolerance=0.0, linear_solver_type=pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG))
    costs = [it["cost"] for it in summ["iterations"]]
    fused = s.eval_fused()
    s.close()
    return step * 1e6, kern * 1e3, costs, fused


def main():
    cfg, reps = sys.argv[1], int(sys.argv[2])
    variants = [parse(a) for a in sys.argv[3:]]
    pkg = _pkgload.load()
    DEFAULT_LIB.append(pkg.load_library())
    prob = pkg.synth(**pkg.CONFIGS[cfg])
    res = {n: [] for n, _ in variants}
    ref = None
    for r in range(reps):
        for n, env in variants:
            step, kern, costs, fused = run(pkg, prob, env)
            if ref is None:
                ref = costs
            dev = max((abs(a - b) / abs(b) for a, b in zip(costs, ref)), default=float("nan"))
            res[n].append((step, kern))
            print(f"rep {r} {n:14s} step {step:7.2f} us  kernel {kern:7.2f} us  sched {fused}  cost dev {dev:.1e}",
                  flush=True)
    print("medians:")
    for n, v in res.items():
        a = np.array(v)
        print(f"  {n:14s} step {np.median(a[:, 0]):7.2f} us  kernel {np.median(a[:, 1]):7.2f} us "
              f"(min {a[:, 1].min():.2f})")


if __name__ == "__main__":
    main()
