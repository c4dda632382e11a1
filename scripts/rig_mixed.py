"""Matrix-free PCG on the C5 rig: fp64 products against the mixed-precision products
(pcg_fp32: fp32 per-observation arithmetic, fp64 sums and true residuals). Per-iteration
wall-clock, costs and CG counts of both, and the oracle's recorded c5_pcg trajectory
(tests/golden/trajectories.json) beside them. Usage: python scripts/rig_mixed.py [iters] [config]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
cfg = sys.argv[2] if len(sys.argv) > 2 else "c5_rig_16x64"
prob = pkg.synth(**pkg.CONFIGS[cfg])
s = pkg.Solver(0)
s.set_problem(prob)
pts0, ext0 = prob.points.copy(), prob.ext.copy()
for name, f32 in (("fp64", 0), ("mixed", 1), ("fp64", 0), ("mixed", 1)):
    s.update_parameters(pts0, ext0)
    t = time.perf_counter()
    r = s.solve(pkg.options(max_num_iterations=iters, function_tolerance=0.0, gradient_tolerance=0.0,
                            parameter_tolerance=0.0, pcg_fp32=f32,
                            linear_solver_type=pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG))
    wall = time.perf_counter() - t
    its = [it["time"] * 1e3 for it in r["iterations"][1:]]
    print(f"{name}: schedule {s.pcg_matrix_free()} wall {wall * 1e3:.1f} ms, iter ms {np.round(its, 3).tolist()}, "
          f"median {np.median(its):.3f}, cg {[it['linear_solver_iterations'] for it in r['iterations'][1:]]}, "
          f"costs {['%.12e' % it['cost'] for it in r['iterations']]}", flush=True)
s.close()
traj = json.load(open(os.path.join(ROOT, "tests", "golden", "trajectories.json")))
for k, v in traj.items():
    if v["config"] == cfg and v["solver"] == "pcg":
        print(f"oracle {k}: cg {v['linear_iterations'][1:]}, costs {['%.12e' % c for c in v['costs']]}")
