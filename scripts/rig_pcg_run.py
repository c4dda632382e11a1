"""One rig (C5) PCG solve, 5 LM iterations, fp64 products (pcg_fp32=0) by default; prints
the per-iteration CG counts, the final cost and the median LM iteration time as JSON. Knobs
come from the environment (e.g. DAB_MF_DIAG), so an A/B runs this once per process.

usage: python scripts/rig_pcg_run.py [CONFIG] [fp32]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
if os.environ.get("DAB_LIB"):  # another build of libdab (A/B)
    abi = sys.modules[pkg.__name__ + "._abi"]
    abi._LIB = abi.load_library(os.path.join(ROOT, os.environ["DAB_LIB"]))
cfg = sys.argv[1] if len(sys.argv) > 1 else "c5_rig_16x64"
f32 = int(sys.argv[2]) if len(sys.argv) > 2 else 0
prob = pkg.synth(**pkg.CONFIGS[cfg])
s = pkg.Solver(0)
s.set_problem(prob)
o = pkg.options(max_num_iterations=5, linear_solver_type=pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG, pcg_fp32=f32)
t0 = time.perf_counter()
r = s.solve(o)
wall = time.perf_counter() - t0
its = [it["time"] for it in r["iterations"][1:]]
print(json.dumps({"cfg": cfg, "fp32": f32, "env": {k: v for k, v in os.environ.items() if k.startswith("DAB_")},
                  "cg": [it["linear_solver_iterations"] for it in r["iterations"][1:]],
                  "final_cost": r["final_cost"], "costs": [it["cost"] for it in r["iterations"]],
                  "iter_ms_median": 1e3 * float(np.median(its)) if its else None, "wall_s": wall}))
s.close()
