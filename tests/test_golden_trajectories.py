"""CPU checks of the committed full-size oracle trajectories (tests/golden/trajectories.json,
oracle/gen_trajectories.py): every record is complete, and the C2 records (the oracle takes
about a second there) are reproduced by rerunning the oracle on the regenerated problem, so
the fixture, the generator and the oracle agree in this container."""
import json
import os

import numpy as np
import pytest

from golden_util import GOLDEN

TRAJ = json.load(open(os.path.join(GOLDEN, "trajectories.json")))
PARAMS = np.load(os.path.join(GOLDEN, "trajectory_params.npz"))


def test_records_cover_the_baseline_configs():
    cfgs = {(r["config"], r["solver"]) for r in TRAJ.values()}
    for c in ("c2_100cam", "c3_1kcam", "c5_rig_16x64"):
        assert (c, "explicit") in cfgs and (c, "pcg") in cfgs
    for r in TRAJ.values():
        assert len(r["costs"]) == r["num_iterations"] + 1 == len(r["success"]) == len(r["gradient_max_norms"])
        assert r["costs"][-1] < r["costs"][0]
    for name, r in TRAJ.items():
        pts = PARAMS[name + "_dpoints32"] if name + "_dpoints32" in PARAMS else PARAMS[name + "_points"]
        assert PARAMS[name + "_ext"].shape[1] == 6 and pts.shape[1] == 3
        # every point recorded (the generated problem's point count)
        assert pts.shape[0] == {"c2_100cam": 10000, "c3_1kcam": 100000, "c5_rig_16x64": 1000000}[r["config"]]
    # the C3 and C5 records cover the LM iterations bench.py times (--lm-iters 5)
    for n in ("c3_explicit", "c3_pcg", "c5_explicit", "c5_pcg"):
        assert TRAJ[n]["max_num_iterations"] == 5
    # full-size records that end by the function tolerance (Ceres defaults), not the cap
    conv = [n for n, r in TRAJ.items() if r.get("converge")]
    assert conv and all(TRAJ[n]["termination"] == "CONVERGENCE" for n in conv)


@pytest.mark.parametrize("name", ["c2_explicit", "c2_pcg", "c2_converge"])
def test_c2_record_reproduces(pkg, orc, name):
    import gen_trajectories as gt
    rec = TRAJ[name]
    prob = pkg.synth(**pkg.CONFIGS[rec["config"]])
    assert gt.problem_digest(prob) == rec["digest"]
    p_init = prob.points.copy()
    o = orc.solve(pkg, prob, gt.record_options(pkg, rec))
    assert o["termination"] == rec["termination"] and o["num_iterations"] == rec["num_iterations"]
    assert [it["linear_solver_iterations"] for it in o["iterations"]] == rec["linear_iterations"]
    for a, b in zip([it["cost"] for it in o["iterations"]], rec["costs"]):
        assert a == pytest.approx(b, rel=1e-12)
    for a, b in zip([it["gradient_max_norm"] for it in o["iterations"]], rec["gradient_max_norms"]):
        assert a == pytest.approx(b, rel=1e-12)
    np.testing.assert_allclose(prob.points, gt.reference_points(PARAMS, name, p_init), rtol=0, atol=1e-12)
    np.testing.assert_allclose(prob.ext, PARAMS[name + "_ext"], rtol=0, atol=1e-12)
