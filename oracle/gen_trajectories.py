"""TEST INFRASTRUCTURE ONLY: oracle LM trajectories of the BASELINE configurations at full
size, committed as tests/golden/trajectories.json (the -m gpu full-size parity tests compare
the HIP path against them; the CPU oracle takes seconds to minutes per iteration at these
sizes, too long to rerun inside a test).

The problems come from libdab's deterministic host generator (dab_synth_fill: splitmix64 /
xoshiro256** streams), so the GPU box regenerates the identical problem; each
record carries a digest of the generated arrays that the tests verify first.

Usage: python oracle/gen_trajectories.py [record ...]   (default: every record below)
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
import _pkgload  # noqa: E402
import oracle  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "trajectories.json")
# final parameters of every record, in tests/golden/trajectory_params.npz: extrinsics in full
# (float64); points in full, as float64 (`_points`) or — the 1M-point rig records — as the
# float32 change from the generated initial points (`_dpoints32`: the change is < 0.1, so
# float32 keeps it to ~1e-9, far inside the 1e-7 / 1e-6 tolerances, at half the size)
PARAMS = os.path.join(ROOT, "tests", "golden", "trajectory_params.npz")
DELTA32 = {"c5_explicit", "c5_pcg"}

# (record name, config, linear solver, LM iterations, converge). Tolerances are zeroed so that
# every iteration runs, as in bench.py — except for the `converge` records, which keep Ceres'
# default tolerances and end by CONVERGENCE (function tolerance) at full size.
CASES = [
    ("c2_explicit", "c2_100cam", "explicit", 4, False),
    ("c2_pcg", "c2_100cam", "pcg", 4, False),
    ("c3_explicit", "c3_1kcam", "explicit", 5, False),
    ("c3_pcg", "c3_1kcam", "pcg", 5, False),
    ("c5_explicit", "c5_rig_16x64", "explicit", 5, False),
    ("c5_pcg", "c5_rig_16x64", "pcg", 5, False),
    ("c2_converge", "c2_100cam", "explicit", 100, True),
    ("c3_converge", "c3_1kcam", "explicit", 100, True),
]


def problem_digest(prob):
    """sha256 over the generated arrays (bit patterns), so the tests know they regenerated
    exactly the problem the trajectory was computed on."""
    h = hashlib.sha256()
    for a in (prob.obs_xy, prob.obs_point, prob.obs_ext0, prob.obs_ext1, prob.obs_intr, prob.points,
              prob.ext, prob.intr, prob.intr_nf, prob.intr_nk, prob.ext_const):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def case_options(pkg, solver, iters, threads=8, converge=False):
    lst = (pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR if solver == "explicit"
           else pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)
    if converge:  # Ceres' default tolerances
        return pkg.options(max_num_iterations=iters, linear_solver_type=lst, num_threads=threads)
    return pkg.options(max_num_iterations=iters, function_tolerance=0.0, gradient_tolerance=0.0,
                       parameter_tolerance=0.0, linear_solver_type=lst, num_threads=threads)


def record_options(pkg, rec, threads=8):
    return case_options(pkg, rec["solver"], rec["max_num_iterations"], threads, rec.get("converge", False))


def reference_points(params, name, initial_points):
    """The oracle's final points of record `name` (every point), float64."""
    if name + "_dpoints32" in params:
        return initial_points + params[name + "_dpoints32"].astype(np.float64)
    return params[name + "_points"]


def sample_rows(a, n):
    return a[:: max(1, a.shape[0] // n)][:n]


def gauge_normalised(points, ext):
    """The reference's gauge fixes one extrinsic only: the scene's scale
    stays free, so two correct solvers may drift apart along it by rounding. Points and
    translations divided by the RMS spread of the points about their centroid; rotations
    unchanged."""
    c = points.mean(axis=0)
    sigma = float(np.sqrt(((points - c) ** 2).sum(axis=1).mean()))
    e = ext.copy()
    e[:, 3:] /= sigma
    return points / sigma, e, sigma


def main(names):
    pkg = _pkgload.load()
    threads = int(os.environ.get("ORACLE_THREADS", min(16, os.cpu_count() or 1)))
    out = json.load(open(OUT)) if os.path.exists(OUT) else {}
    params = dict(np.load(PARAMS)) if os.path.exists(PARAMS) else {}
    probs = {}
    for name, cfg, solver, iters, converge in CASES:
        if names and name not in names:
            continue
        if cfg not in probs:
            probs = {cfg: pkg.synth(**pkg.CONFIGS[cfg])}
        prob = probs[cfg].copy()
        digest = problem_digest(prob)
        p_init = prob.points.copy()
        t = time.perf_counter()
        o = oracle.solve(pkg, prob, case_options(pkg, solver, iters, threads, converge))
        wall = time.perf_counter() - t
        out[name] = dict(
            config=cfg, solver=solver, max_num_iterations=iters, digest=digest, num_obs=prob.num_obs,
            termination=o["termination"], num_iterations=o["num_iterations"],
            costs=[it["cost"] for it in o["iterations"]],
            success=[bool(it["success"]) for it in o["iterations"]],
            linear_iterations=[it["linear_solver_iterations"] for it in o["iterations"]],
            final_cost=o["final_cost"],
            gradient_max_norms=[it["gradient_max_norm"] for it in o["iterations"]],
            step_norms=[it["step_norm"] for it in o["iterations"]],
            trust_region_radii=[it["trust_region_radius"] for it in o["iterations"]],
            converge=converge, oracle_wall_s=wall, oracle_threads=threads)
        for k in (name + "_points", name + "_dpoints32"):
            params.pop(k, None)
        if name in DELTA32:
            params[name + "_dpoints32"] = np.ascontiguousarray((prob.points - p_init).astype(np.float32))
        else:
            params[name + "_points"] = np.ascontiguousarray(prob.points)
        params[name + "_ext"] = np.ascontiguousarray(prob.ext)
        print(f"{name}: {o['num_iterations']} its, costs {out[name]['costs']}, "
              f"cg {out[name]['linear_iterations']}, {wall:.1f} s", flush=True)
        with open(OUT, "w") as f:
            json.dump(out, f, indent=1)
        np.savez_compressed(PARAMS, **params)


if __name__ == "__main__":
    main(sys.argv[1:])
