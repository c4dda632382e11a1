"""CPU checks of the committed full-size oracle trajectories (tests/golden/trajectories.json,
oracle/gen_trajectories.py): every record is complete, and the C2 records (the oracle takes
about a second there) are reproduced by rerunning the oracle on the regenerated problem, so
the fixture, the generator and the oracle agree in this container."""
import json
import os

import pytest

from golden_util import GOLDEN

TRAJ = json.load(open(os.path.join(GOLDEN, "trajectories.json")))


def test_records_cover_the_baseline_configs():
    cfgs = {(r["config"], r["solver"]) for r in TRAJ.values()}
    for c in ("c2_100cam", "c3_1kcam", "c5_rig_16x64"):
        assert (c, "explicit") in cfgs and (c, "pcg") in cfgs
    for r in TRAJ.values():
        assert len(r["costs"]) == r["num_iterations"] + 1 == len(r["success"])
        assert r["costs"][-1] < r["costs"][0]


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
