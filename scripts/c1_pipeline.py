"""Config 1's sfm.cc pipeline (runPipeline over libdab) with the per-stage breakdown of
dam_pipeline_report, a few repetitions, and the set-up / first-solve timing of one handle.

usage: python scripts/c1_pipeline.py [reps]
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import _pkgload  # noqa: E402

pkg = _pkgload.load()
import gen_deeparc_fixtures as gen  # noqa: E402
from importlib import import_module  # noqa: E402

host = import_module(pkg.__name__ + ".host_api")
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
pprob = pkg.synth(**dict(pkg.CONFIGS["c1_rig_8x36"], pixel_noise=3.0))
with tempfile.TemporaryDirectory() as td:
    path = os.path.join(td, "c1.deeparc")
    with open(path, "w") as f:
        f.write(gen.problem_to_deeparc(pprob, True, 8, 36, [3, 4, 9], np.random.default_rng(1)))
    for r in range(reps):
        t = time.perf_counter()
        rep = host.run_pipeline_report(path, max_iteration=100, quiet=True)
        wall = time.perf_counter() - t
        bd = {k: round(1e3 * v, 2) for k, v in rep["breakdown"].items()}
        print(json.dumps({"rep": r, "wall_ms": round(1e3 * wall, 2), "total_ms": round(1e3 * rep["total_seconds"], 2),
                          "solves": rep["solves"], "lm_iterations": rep["lm_iterations"], "rounds": rep["rounds"],
                          "points": rep["points"], "final_cost": rep["final_cost"], "breakdown_ms": bd}), flush=True)
# one handle: set-up and first solve of the config-1 problem, then a warm re-solve
c1 = pkg.synth(**pkg.CONFIGS["c1_rig_8x36"])
o1 = pkg.options(max_num_iterations=10)
for rep in range(2):
    tc = time.perf_counter()
    s = pkg.Solver(0)
    t0 = time.perf_counter()
    s.set_problem(c1.copy())
    t1 = time.perf_counter()
    g = s.solve(o1)
    t2 = time.perf_counter()
    s.close()
    t3 = time.perf_counter()
    print(json.dumps({"create_ms": round(1e3 * (t0 - tc), 2), "set_problem_ms": round(1e3 * (t1 - t0), 2),
                      "first_solve_ms": round(1e3 * (t2 - t1), 2), "destroy_ms": round(1e3 * (t3 - t2), 2),
                      "lm_ms": round(1e3 * g["total_time"], 2) if "total_time" in g else None,
                      "iterations": g["num_iterations"]}), flush=True)
