"""One EXPLICIT (DENSE_SCHUR) solve of a config, 5 LM iterations, on a handle whose first
solve (table build, graph capture) ran before; prints the costs and the median LM iteration
time as JSON (DAB_LIB: another build of libdab, for A/Bs).

usage: python scripts/explicit_run.py [CONFIG]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
if os.environ.get("DAB_LIB"):  # another build of libdab (A/B)
    abi = sys.modules[pkg.__name__ + "._abi"]
    abi._LIB = abi.load_library(os.path.join(ROOT, os.environ["DAB_LIB"]))
cfg = sys.argv[1] if len(sys.argv) > 1 else "c3_1kcam"
prob = pkg.synth(**pkg.CONFIGS[cfg])
s = pkg.Solver(0)
o = pkg.options(max_num_iterations=5, linear_solver_type=pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR)
s.set_problem(prob.copy())
s.solve(o)  # warm: tables, captured graph
s.set_problem(prob.copy())
r = s.solve(o)
its = [it["time"] for it in r["iterations"][1:]]
print(json.dumps({"cfg": cfg, "lib": os.environ.get("DAB_LIB", "in-tree"), "final_cost": r["final_cost"],
                  "costs": [it["cost"] for it in r["iterations"]],
                  "iter_ms_median": 1e3 * float(np.median(its)) if its else None}))
s.close()
