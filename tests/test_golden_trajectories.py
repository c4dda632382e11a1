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
        assert PARAMS[name + "_ext"].shape[1] == 6 and PARAMS[name + "_points"].shape[1] == 3
    # the C3 records cover the LM iterations bench.py times (--lm-iters 5)
    assert TRAJ["c3_explicit"]["max_num_iterations"] == TRAJ["c3_pcg"]["max_num_iterations"] == 5


@pytest.mark.parametrize("name", ["c2_explicit", "c2_pcg"])
def test_c2_record_reproduces(pkg, orc, name):
    import gen_trajectories as gt
    rec = TRAJ[name]
    prob = pkg.synth(**pkg.CONFIGS[rec["config"]])
    assert gt.problem_digest(prob) == rec["digest"]
    o = orc.solve(pkg, prob, gt.case_options(pkg, rec["solver"], rec["max_num_iterations"]))
    assert [it["linear_solver_iterations"] for it in o["iterations"]] == rec["linear_iterations"]
    for a, b in zip([it["cost"] for it in o["iterations"]], rec["costs"]):
        assert a == pytest.approx(b, rel=1e-12)
    for a, b in zip([it["gradient_max_norm"] for it in o["iterations"]], rec["gradient_max_norms"]):
        assert a == pytest.approx(b, rel=1e-12)
    np.testing.assert_allclose(prob.points[:: rec["point_stride"]], PARAMS[name + "_points"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(prob.ext, PARAMS[name + "_ext"], rtol=0, atol=1e-12)
