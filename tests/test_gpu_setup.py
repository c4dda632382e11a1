"""dab_set_problem on the device (csrc/dab_setup.hip: rocPRIM stable radix sorts, scans and
gather passes) against the host reference path (DAB_SETUP_HOST=1, the counting sorts of
dab_solver.hip's setup_host). The layouts decide every summation order of the solver, so
the two paths must give bitwise-identical LM trajectories (costs, CG counts, parameters),
residuals and filter masks on every problem shape: BAL, rig (composed observations, pair
chunks, runs of one point on one camera), frozen cameras, unreferenced points and
extrinsics, several chunks per camera."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _problems(pkg):
    out = {
        "bal": pkg.synth(kind=0, num_cameras=40, num_points=3000, obs_per_point=6, seed=71),
        "rig": pkg.synth(kind=1, num_arcs=5, num_rings=12, num_points=2500, obs_per_point=7, seed=72),
        "c2": pkg.synth(**pkg.CONFIGS["c2_100cam"]),
    }
    # unreferenced points and extrinsics, a second gauge camera, observations out of order
    p = pkg.synth(kind=0, num_cameras=30, num_points=2000, obs_per_point=5, seed=73)
    keep = np.ones(p.num_obs, bool)
    keep[p.obs_point % 7 == 3] = False        # points 3, 10, ... unreferenced
    keep[p.obs_ext0 == 11] = False            # extrinsic 11 unreferenced
    rng = np.random.default_rng(5)
    idx = np.nonzero(keep)[0]
    rng.shuffle(idx)
    q = p.subset(idx)
    q.ext_const[4] = 1
    out["holes"] = q
    return out


def _run(pkg, prob, host, monkeypatch, lst, freeze=False, chunk=None, xchunk=None):
    monkeypatch.setenv("DAB_SETUP_HOST", "1" if host else "0")
    for name, val in (("DAB_CHUNK", chunk), ("DAB_XCHUNK", xchunk)):
        if val:
            monkeypatch.setenv(name, str(val))
        else:
            monkeypatch.delenv(name, raising=False)
    p = prob.copy()
    p.freeze_camera = 1 if freeze else 0
    s = pkg.Solver(0)
    try:
        s.set_problem(p)
        r0, c0 = s.residuals()
        g = s.solve(pkg.options(max_num_iterations=6, linear_solver_type=lst))
        r1, c1 = s.residuals()
    finally:
        s.close()
    return g, p, (r0, c0, r1, c1)


@pytest.mark.parametrize("name", ["bal", "rig", "c2", "holes"])
@pytest.mark.parametrize("solver", ["explicit", "pcg"])
def test_device_setup_matches_host_setup(pkg, gpu, monkeypatch, name, solver):
    prob = _problems(pkg)[name]
    lst = pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR if solver == "explicit" else pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG
    a, pa, ra = _run(pkg, prob, False, monkeypatch, lst)
    b, pb, rb = _run(pkg, prob, True, monkeypatch, lst)
    assert [it["cost"] for it in a["iterations"]] == [it["cost"] for it in b["iterations"]]
    assert [it["linear_solver_iterations"] for it in a["iterations"]] == \
        [it["linear_solver_iterations"] for it in b["iterations"]]
    np.testing.assert_array_equal(pa.points, pb.points)
    np.testing.assert_array_equal(pa.ext, pb.ext)
    for x, y in zip(ra, rb):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("name", ["rig", "holes"])
def test_device_setup_small_chunks_and_freeze(pkg, gpu, monkeypatch, name):
    """Several chunks per camera (DAB_CHUNK = 64) and the frozen-camera problem."""
    prob = _problems(pkg)[name]
    for freeze, chunk in ((False, 64), (True, None)):
        a, pa, _ = _run(pkg, prob, False, monkeypatch, pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR, freeze, chunk)
        b, pb, _ = _run(pkg, prob, True, monkeypatch, pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR, freeze, chunk)
        assert [it["cost"] for it in a["iterations"]] == [it["cost"] for it in b["iterations"]]
        np.testing.assert_array_equal(pa.points, pb.points)


def test_device_setup_filter_masks(pkg, gpu, monkeypatch):
    prob = _problems(pkg)["rig"]
    masks = []
    for host in (False, True):
        monkeypatch.setenv("DAB_SETUP_HOST", "1" if host else "0")
        s = pkg.Solver(0)
        try:
            s.set_problem(prob.copy())
            masks.append(s.filter(5.0, [0.0, 0.0, 0.0], 1e6))
        finally:
            s.close()
    for x, y in zip(masks[0], masks[1]):
        np.testing.assert_array_equal(x, y)


def test_device_setup_rejects_bad_index(pkg, gpu, monkeypatch):
    monkeypatch.setenv("DAB_SETUP_HOST", "0")
    p = pkg.synth(kind=0, num_cameras=10, num_points=200, obs_per_point=4, seed=3)
    p.obs_point[17] = p.points.shape[0]  # out of range
    s = pkg.Solver(0)
    try:
        with pytest.raises(RuntimeError, match="observation 17"):
            s.set_problem(p)
    finally:
        s.close()


def test_pair_chunks_cut_into_pieces(pkg, gpu, monkeypatch):
    """Pairs cut into several equal pieces (DAB_XCHUNK = 100: every pair of this rig spans
    several k_eval_pair chunks): device and host set-up agree bitwise, and the trajectory
    stays within rounding of the one-chunk-per-pair layout."""
    prob = _problems(pkg)["rig"]
    lst = pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR
    a, pa, _ = _run(pkg, prob, False, monkeypatch, lst, xchunk=100)
    b, pb, _ = _run(pkg, prob, True, monkeypatch, lst, xchunk=100)
    c, pc, _ = _run(pkg, prob, False, monkeypatch, lst)
    assert [it["cost"] for it in a["iterations"]] == [it["cost"] for it in b["iterations"]]
    np.testing.assert_array_equal(pa.points, pb.points)
    ca, cc = [it["cost"] for it in a["iterations"]], [it["cost"] for it in c["iterations"]]
    assert len(ca) == len(cc)
    np.testing.assert_allclose(ca, cc, rtol=1e-12)


@pytest.mark.parametrize("host", [False, True])
def test_pair_eval_mixed_intrinsics(pkg, gpu, monkeypatch, host):
    """k_eval_pair reads a chunk's arc, ring and intrinsic tables once when every record of
    an (arc, ring) pair names one intrinsic (the rig: intrinsic = arc). Here intrinsic 0 is
    duplicated and every other observation of it re-pointed at the copy, so pairs mix two
    intrinsics of equal values: the set-up must fall back to per-record tables, and the
    trajectory must equal the unmodified problem's bitwise (same values, same sums)."""
    prob = _problems(pkg)["rig"]
    q = prob.copy()
    ni = q.intr.shape[0]
    q.intr = np.ascontiguousarray(np.vstack([q.intr, q.intr[:1]]))
    q.intr_nf = np.ascontiguousarray(np.append(q.intr_nf, q.intr_nf[0]).astype(np.int32))
    q.intr_nk = np.ascontiguousarray(np.append(q.intr_nk, q.intr_nk[0]).astype(np.int32))
    sel = np.nonzero(q.obs_intr == 0)[0][::2]
    assert len(sel) > 0
    q.obs_intr[sel] = ni
    for lst in (pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR, pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG):
        a, pa, ra = _run(pkg, prob, host, monkeypatch, lst)
        b, pb, rb = _run(pkg, q, host, monkeypatch, lst)
        assert [it["cost"] for it in a["iterations"]] == [it["cost"] for it in b["iterations"]]
        assert [it["linear_solver_iterations"] for it in a["iterations"]] == \
            [it["linear_solver_iterations"] for it in b["iterations"]]
        np.testing.assert_array_equal(pa.points, pb.points)
        np.testing.assert_array_equal(pa.ext, pb.ext)
