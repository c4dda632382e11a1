"""HIP path (libdab.so via the C ABI) vs the CPU oracle and the golden vectors.

Tolerances (fp64, stated): residuals 1e-12 relative (to max(1,|r|)); Jacobians 1e-11
relative to the case's largest entry against the golden vectors (everywhere, including
Ceres' near-branch regime), 1e-9 against the oracle's autodiff on synthetic problems;
LM trajectories: per-iteration cost 1e-9 relative, same iteration count and termination,
final parameters 1e-7 absolute (they are O(1)).
"""
import numpy as np
import pytest

from golden_util import TOL_JAC, TOL_RES, cases_problem, functor_cases, golden_arrays

pytestmark = pytest.mark.gpu


def gpu_jac(pkg, prob):
    s = pkg.Solver(0)
    try:
        s.set_problem(prob)
        return s.jacobians()
    finally:
        s.close()


def test_jacobian_kernel_vs_golden(pkg, gpu):
    cases = functor_cases()
    r, J = gpu_jac(pkg, cases_problem(pkg, cases))
    rg, Jg = golden_arrays(cases)
    for i, c in enumerate(cases):
        er = np.abs(r[i] - rg[i]).max() / max(1.0, np.abs(rg[i]).max())
        assert er < TOL_RES, (i, c["regime"], er)
        eJ = np.abs(J[i] - Jg[i]).max() / np.abs(Jg[i]).max()
        assert eJ < TOL_JAC, (i, c["regime"], c["compose"], c["nf"], c["nk"], eJ)


@pytest.mark.parametrize("kind", ["bal", "rig"])
def test_jacobian_kernel_vs_oracle(pkg, orc, gpu, kind):
    if kind == "bal":
        prob = pkg.synth(kind=0, num_cameras=40, num_points=3000, obs_per_point=7, seed=5)
    else:
        prob = pkg.synth(kind=1, num_arcs=5, num_rings=12, num_points=3000, obs_per_point=7, seed=6)
    r, J = gpu_jac(pkg, prob)
    ro, Jo = orc.eval_jacobians(pkg, prob)
    np.testing.assert_allclose(r, ro, rtol=0, atol=1e-12 * max(1.0, np.abs(ro).max()))
    scale = np.abs(Jo).reshape(len(Jo), -1).max(axis=1)
    err = np.abs(J - Jo).reshape(len(Jo), -1).max(axis=1) / scale
    assert err.max() < 1e-9, err.max()


def test_rotations_near_pi_match_oracle(pkg, orc, gpu):
    """cam_table's power series for sin(th)/th, (1-cos th)/th^2 and (th-sin th)/th^3 runs up
    to |w| = pi, where sin(th)/th -> 0 and the alternating series cancels terms of ~3.7. Camera
    rotations with |w| in [2.5, pi) (and a few just above pi: the closed form), every
    observation in front of its camera: the residuals and Jacobians (k_jacobian_full) against
    the oracle's Ceres-equivalent AngleAxisRotatePoint + autodiff, and the LM trajectory through
    the fused evaluation pass (whose tables are built in-kernel by the same series)."""
    base = pkg.synth(kind=0, num_cameras=48, num_points=3000, obs_per_point=6, seed=77)
    rng = np.random.default_rng(77)
    for e in range(base.ext.shape[0]):
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        th = rng.uniform(2.5, np.pi - 1e-6) if e % 8 else rng.uniform(np.pi, np.pi + 0.05)
        base.ext[e, :3] = d * th
        base.ext[e, 3:] = [rng.normal(scale=0.05), rng.normal(scale=0.05), 2.0]  # points at depth ~2
    prob = base.copy()
    r, _ = orc.eval_residuals(pkg, prob)
    prob.obs_xy += r  # observe the projection, then 1 px noise and perturbed points
    prob.obs_xy += rng.normal(size=prob.obs_xy.shape)
    prob.points += rng.normal(scale=1e-3, size=prob.points.shape)
    th = np.linalg.norm(prob.ext[:, :3], axis=1)
    assert th.min() > 2.5 and (th < np.pi).sum() >= 40 and (th > np.pi).sum() >= 1
    rg, J = gpu_jac(pkg, prob.copy())
    ro, Jo = orc.eval_jacobians(pkg, prob)
    np.testing.assert_allclose(rg, ro, rtol=0, atol=1e-12 * max(1.0, np.abs(ro).max()))
    scale = np.abs(Jo).reshape(len(Jo), -1).max(axis=1)
    err = np.abs(J - Jo).reshape(len(Jo), -1).max(axis=1) / scale
    assert err.max() < 1e-9, err.max()
    g, o, ref = run_both(pkg, orc, prob, max_num_iterations=10)
    assert_same_trajectory(g, o, prob, ref)


def test_residual_pass_vs_oracle(pkg, orc, gpu):
    prob = pkg.synth(kind=1, num_arcs=4, num_rings=9, num_points=2000, obs_per_point=6, seed=8)
    s = pkg.Solver(0)
    try:
        s.set_problem(prob)
        r, cost = s.residuals()
    finally:
        s.close()
    ro, co = orc.eval_residuals(pkg, prob)
    np.testing.assert_allclose(r, ro, rtol=0, atol=1e-12 * np.abs(ro).max())
    assert cost == pytest.approx(co, rel=1e-12)


def run_both(pkg, orc, prob, **kw):
    ref = prob.copy()
    opts = pkg.options(num_threads=8, **kw)
    s = pkg.Solver(0)
    try:
        s.set_problem(prob)
        g = s.solve(opts)
    finally:
        s.close()
    o = orc.solve(pkg, ref, opts)
    return g, o, ref


def assert_same_trajectory(g, o, prob, ref, tol_cost=1e-9, tol_x=1e-7):
    assert g["termination"] == o["termination"], (g["message"], o["message"])
    assert g["num_iterations"] == o["num_iterations"]
    assert len(g["iterations"]) == len(o["iterations"])
    for a, b in zip(g["iterations"], o["iterations"]):
        assert a["success"] == b["success"]
        assert abs(a["cost"] - b["cost"]) <= tol_cost * abs(b["cost"]), (a, b)
    assert g["initial_cost"] == pytest.approx(o["initial_cost"], rel=1e-12)
    assert g["final_cost"] == pytest.approx(o["final_cost"], rel=tol_cost)
    assert np.abs(prob.points - ref.points).max() < tol_x
    assert np.abs(prob.ext - ref.ext).max() < tol_x


def test_lm_bal_matches_oracle(pkg, orc, gpu):
    prob = pkg.synth(kind=0, num_cameras=60, num_points=4000, obs_per_point=6, seed=21)
    g, o, ref = run_both(pkg, orc, prob, max_num_iterations=30)
    assert_same_trajectory(g, o, prob, ref)
    assert g["final_cost"] < 0.02 * g["initial_cost"]


@pytest.mark.parametrize("solver", ["explicit", "pcg"])
def test_lm_bal_ragged_matches_oracle(pkg, orc, gpu, solver):
    """Ragged tracks (2..12 observations per point, so SELL slices carry padding slots and
    the camera chunks differ in length) through the fused evaluation pass and both
    linear solvers, against the oracle's trajectory. Two points of one observation are
    kept (their V block is rank deficient until damped)."""
    base = pkg.synth(kind=0, num_cameras=80, num_points=5000, obs_per_point=12, seed=61)
    rng = np.random.default_rng(61)
    keep_n = rng.integers(2, 13, size=base.points.shape[0])
    keep_n[:2] = 1
    rank_in_track = np.zeros(base.num_obs, np.int64)
    order = np.argsort(base.obs_point, kind="stable")
    pts = base.obs_point[order]
    first = np.r_[0, np.flatnonzero(np.diff(pts)) + 1]
    start = np.repeat(first, np.diff(np.r_[first, len(pts)]))
    rank_in_track[order] = np.arange(len(pts)) - start
    prob = base.subset(rank_in_track < keep_n[base.obs_point]).copy()
    lst = (pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR if solver == "explicit"
           else pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)
    g, o, ref = run_both(pkg, orc, prob, max_num_iterations=20, linear_solver_type=lst)
    assert_same_trajectory(g, o, prob, ref, tol_cost=1e-9 if solver == "explicit" else 1e-8)


def test_lm_rig_matches_oracle(pkg, orc, gpu):
    prob = pkg.synth(kind=1, num_arcs=6, num_rings=16, num_points=3000, obs_per_point=8, seed=22)
    assert (prob.obs_ext1 >= 0).any() and (prob.obs_ext1 < 0).any()
    g, o, ref = run_both(pkg, orc, prob, max_num_iterations=30)
    assert_same_trajectory(g, o, prob, ref)


def test_lm_rig_large_tables_matches_oracle(pkg, orc, gpu):
    """A rig whose extrinsic / intrinsic tables exceed the LDS staging limit (E > 128): the
    camera-side and cross-block passes read the tables from global memory and the
    pair-major pass is off. Against the oracle's trajectory."""
    prob = pkg.synth(kind=1, num_arcs=9, num_rings=122, num_points=2500, obs_per_point=6, seed=23)
    assert prob.ext.shape[0] > 128 and (prob.obs_ext1 >= 0).any()
    g, o, ref = run_both(pkg, orc, prob, max_num_iterations=12)
    assert_same_trajectory(g, o, prob, ref)


@pytest.mark.parametrize("solver", ["explicit", "pcg"])
def test_rig_pair_eval_matches_camera_major(pkg, gpu, solver, monkeypatch):
    """The rig's composed observations evaluated pair-major (k_eval_pair: both cameras'
    blocks and the cross block from one projection, rotated frame) against the
    camera-major + cross passes (DAB_PAIR_EVAL=0): same LM trajectory to 1e-10 relative,
    same CG counts; the pair-major pass is bitwise repeatable."""
    prob = pkg.synth(kind=1, num_arcs=6, num_rings=16, num_points=3000, obs_per_point=8, seed=24)
    lst = (pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR if solver == "explicit"
           else pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)
    res, pts = [], []
    for pe in ("1", "0", "1"):
        monkeypatch.setenv("DAB_PAIR_EVAL", pe)
        p = prob.copy()
        s = pkg.Solver(0)
        s.set_problem(p)
        res.append(s.solve(pkg.options(max_num_iterations=10, linear_solver_type=lst)))
        s.close()
        pts.append(p.points.copy())
    a, b = res[0], res[1]
    assert [it["linear_solver_iterations"] for it in a["iterations"]] == \
        [it["linear_solver_iterations"] for it in b["iterations"]]
    np.testing.assert_allclose([it["cost"] for it in a["iterations"]], [it["cost"] for it in b["iterations"]],
                               rtol=1e-10)
    np.testing.assert_array_equal(pts[0], pts[2])


@pytest.mark.parametrize("kind", ["bal", "rig"])
def test_lm_pcg_matches_oracle(pkg, orc, gpu, kind):
    """IMPLICIT_SCHUR_PCG: the GPU implicit operator vs the oracle's CG on the explicit S.
    Same recurrences; only summation order differs, so CG iteration counts and the LM
    trajectory agree (costs 1e-8 relative)."""
    if kind == "bal":
        prob = pkg.synth(kind=0, num_cameras=50, num_points=3000, obs_per_point=6, seed=31)
    else:
        prob = pkg.synth(kind=1, num_arcs=6, num_rings=14, num_points=2500, obs_per_point=8, seed=32)
    g, o, ref = run_both(pkg, orc, prob, max_num_iterations=15,
                         linear_solver_type=pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)
    assert_same_trajectory(g, o, prob, ref, tol_cost=1e-8, tol_x=1e-6)
    gi = [it["linear_solver_iterations"] for it in g["iterations"]]
    oi = [it["linear_solver_iterations"] for it in o["iterations"]]
    assert gi == oi
    assert max(gi) > 1
    assert g["final_cost"] < 0.05 * g["initial_cost"]


def test_lm_pcg_reaches_dense_schur_minimum(pkg, gpu):
    prob = pkg.synth(kind=1, num_arcs=5, num_rings=12, num_points=2000, obs_per_point=7, seed=33)
    res = []
    for lst in (pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR, pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG):
        p = prob.copy()
        s = pkg.Solver(0)
        s.set_problem(p)
        res.append(s.solve(pkg.options(max_num_iterations=50, linear_solver_type=lst))["final_cost"])
        s.close()
    assert res[1] == pytest.approx(res[0], rel=1e-4)


@pytest.mark.parametrize("kind", ["bal", "rig"])
def test_lm_pcg_fp32_reaches_same_minimum(pkg, gpu, kind, monkeypatch):
    """Mixed-precision PCG (fp32 Schur factors Y, fp64 everything else): the same LM
    reaches the fp64 minimum (final cost 1e-6 relative); its CG iteration counts may
    differ, so only the endpoint is compared. (Small camera sets default to the
    matrix-free PCG, which stores no Y; DAB_PCG_MF=0 keeps the stored-Y path here.)"""
    monkeypatch.setenv("DAB_PCG_MF", "0")
    if kind == "bal":
        prob = pkg.synth(kind=0, num_cameras=50, num_points=3000, obs_per_point=6, seed=34)
    else:
        prob = pkg.synth(kind=1, num_arcs=6, num_rings=14, num_points=2500, obs_per_point=8, seed=35)
    res = []
    for f32 in (0, 1):
        p = prob.copy()
        s = pkg.Solver(0)
        s.set_problem(p)
        res.append(s.solve(pkg.options(max_num_iterations=50, pcg_fp32=f32,
                                       linear_solver_type=pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)))
        s.close()
    assert res[1]["final_cost"] == pytest.approx(res[0]["final_cost"], rel=1e-6)
    assert res[1]["termination"] == "CONVERGENCE"


@pytest.mark.parametrize("kind", ["bal", "rig"])
def test_pcg_fused_matvec_matches_two_pass(pkg, gpu, kind, monkeypatch):
    """Small camera systems use the single-pass S*p (per-wave LDS camera accumulators);
    DAB_PCG_FUSED=0 forces the camera-major + point-major passes. Both must give the same
    LM trajectory: per-iteration cost 1e-9 relative and the same CG iteration counts
    (only the summation order of S*p differs). The fused one must be bitwise repeatable."""
    if kind == "bal":
        prob = pkg.synth(kind=0, num_cameras=60, num_points=4000, obs_per_point=7, seed=41)
    else:
        prob = pkg.synth(kind=1, num_arcs=6, num_rings=16, num_points=3000, obs_per_point=8, seed=42)
    monkeypatch.setenv("DAB_PCG_MF", "0")  # the stored-Y products (the matrix-free PCG has its own test)
    opts = dict(max_num_iterations=15, linear_solver_type=pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)
    res, pts = [], []
    for fused in ("1", "0", "1"):
        monkeypatch.setenv("DAB_PCG_FUSED", fused)
        p = prob.copy()
        s = pkg.Solver(0)
        s.set_problem(p)
        res.append(s.solve(pkg.options(**opts)))
        s.close()
        pts.append(p.points.copy())
    a, b = res[0], res[1]
    assert [it["linear_solver_iterations"] for it in a["iterations"]] == \
        [it["linear_solver_iterations"] for it in b["iterations"]]
    np.testing.assert_allclose([it["cost"] for it in a["iterations"]], [it["cost"] for it in b["iterations"]],
                               rtol=1e-9)
    np.testing.assert_array_equal(pts[0], pts[2])  # fused path: bitwise repeatable


@pytest.mark.parametrize("kind", ["bal", "rig"])
def test_matrix_free_pcg_matches_stored_y(pkg, gpu, kind, monkeypatch):
    """Small camera sets run the PCG matrix-free (Y_e re-evaluated in every pass: diagonal
    blocks and rhs, products, back substitution). DAB_PCG_MF=0 stores the fp64 Y records
    instead. Same LM trajectory: cost 1e-9 relative, same CG iteration counts (only the
    association of the Schur products differs); the matrix-free path is bitwise
    repeatable."""
    if kind == "bal":
        prob = pkg.synth(kind=0, num_cameras=60, num_points=4000, obs_per_point=7, seed=45)
    else:
        prob = pkg.synth(kind=1, num_arcs=6, num_rings=16, num_points=3000, obs_per_point=8, seed=46)
    opts = dict(max_num_iterations=15, linear_solver_type=pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)
    res, pts = [], []
    for mf in ("1", "0", "1"):
        monkeypatch.setenv("DAB_PCG_MF", mf)
        p = prob.copy()
        s = pkg.Solver(0)
        s.set_problem(p)
        res.append(s.solve(pkg.options(**opts)))
        s.close()
        pts.append(p.points.copy())
    a, b = res[0], res[1]
    assert [it["linear_solver_iterations"] for it in a["iterations"]] == \
        [it["linear_solver_iterations"] for it in b["iterations"]]
    np.testing.assert_allclose([it["cost"] for it in a["iterations"]], [it["cost"] for it in b["iterations"]],
                               rtol=1e-9)
    np.testing.assert_array_equal(pts[0], pts[2])


@pytest.mark.parametrize("kind", ["bal", "rig"])
def test_matrix_free_mixed_precision_pcg_matches_oracle(pkg, orc, gpu, kind):
    """BASELINE config 5's mixed-precision PCG where the products are matrix-free (small
    camera sets, the rig): pcg_fp32 runs the Schur products with fp32 per-observation
    arithmetic (k_mf_frame32) and keeps the sums, the CG recurrences and the true residual
    r = b - S x of every 10th CG iteration in fp64 (the refinement step). Against the oracle's
    fp64 CG trajectory: identical CG iteration counts and termination, per-iteration cost
    within 1e-6 relative (the fp32 products perturb each step at ~1e-7), points within 1e-5.
    The run reports the mixed schedule."""
    if kind == "bal":
        prob = pkg.synth(kind=0, num_cameras=60, num_points=4000, obs_per_point=7, seed=61)
    else:
        prob = pkg.synth(kind=1, num_arcs=6, num_rings=16, num_points=3000, obs_per_point=8, seed=62)
    opts = pkg.options(max_num_iterations=12, pcg_fp32=1, num_threads=8,
                       linear_solver_type=pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)
    ref = prob.copy()
    s = pkg.Solver(0)
    try:
        s.set_problem(prob)
        g = s.solve(opts)
        assert s.pcg_matrix_free() == 2 and g["schur_assembly"] == 2
    finally:
        s.close()
    o = orc.solve(pkg, ref, opts)
    assert g["termination"] == o["termination"] and len(g["iterations"]) == len(o["iterations"])
    assert [it["linear_solver_iterations"] for it in g["iterations"]] == \
        [it["linear_solver_iterations"] for it in o["iterations"]]
    dev = 0.0
    for a, b in zip(g["iterations"], o["iterations"]):
        assert a["success"] == b["success"]
        dev = max(dev, abs(a["cost"] - b["cost"]) / abs(b["cost"]))
    print(f"mixed-precision PCG vs oracle fp64 CG: max relative cost deviation {dev:.2e}, "
          f"max |dX| {np.abs(prob.points - ref.points).max():.2e}")
    assert dev <= 1e-6
    np.testing.assert_allclose(prob.points, ref.points, rtol=0, atol=1e-5)


@pytest.mark.parametrize("kind", ["bal", "rig"])
def test_cg_update_work_groups_match_single(pkg, gpu, kind, monkeypatch):
    """The CG update spread over work-groups (last-arriver grid sums) against the
    single-work-group kernel (DAB_CG_ONEWG=1): same CG iteration counts, costs 1e-10."""
    if kind == "bal":
        prob = pkg.synth(kind=0, num_cameras=300, num_points=6000, obs_per_point=6, seed=43)
    else:
        prob = pkg.synth(kind=1, num_arcs=6, num_rings=16, num_points=3000, obs_per_point=8, seed=44)
    res = []
    for one in ("1", "0"):
        monkeypatch.setenv("DAB_CG_ONEWG", one)
        p = prob.copy()
        s = pkg.Solver(0)
        s.set_problem(p)
        res.append(s.solve(pkg.options(max_num_iterations=12,
                                       linear_solver_type=pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)))
        s.close()
    a, b = res
    assert [it["linear_solver_iterations"] for it in a["iterations"]] == \
        [it["linear_solver_iterations"] for it in b["iterations"]]
    np.testing.assert_allclose([it["cost"] for it in a["iterations"]], [it["cost"] for it in b["iterations"]],
                               rtol=1e-10)


@pytest.mark.parametrize("solver", ["explicit", "pcg"])
def test_fused_eval_matches_two_kernel_pass(pkg, gpu, solver, monkeypatch):
    """BAL-shaped problems evaluate in one fused launch (camera and point waves side by
    side, fixed-point cost); DAB_EVAL_FUSED=0 forces the two-kernel pass. The LM
    trajectories must agree (cost 1e-10 relative, same iteration and CG counts; V, g and
    the cost are summed in the same order, U, g_c regrouped), and the fused pass must be
    bitwise repeatable."""
    prob = pkg.synth(kind=0, num_cameras=120, num_points=9000, obs_per_point=8, seed=51)
    lst = (pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR if solver == "explicit"
           else pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)
    res, pts = [], []
    for fused in ("1", "0", "1"):
        monkeypatch.setenv("DAB_EVAL_FUSED", fused)
        p = prob.copy()
        s = pkg.Solver(0)
        s.set_problem(p)
        res.append(s.solve(pkg.options(max_num_iterations=12, linear_solver_type=lst)))
        s.close()
        pts.append(p.points.copy())
    a, b = res[0], res[1]
    assert len(a["iterations"]) == len(b["iterations"]) and a["termination"] == b["termination"]
    assert [it["linear_solver_iterations"] for it in a["iterations"]] == \
        [it["linear_solver_iterations"] for it in b["iterations"]]
    np.testing.assert_allclose([it["cost"] for it in a["iterations"]], [it["cost"] for it in b["iterations"]],
                               rtol=1e-10)
    np.testing.assert_array_equal(pts[0], pts[2])


@pytest.mark.parametrize("shape", [(1024, 20000, 6), (300, 8000, 6), (33, 3000, 5), (2, 700, 2)])
def test_fused_eval_edge_shapes(pkg, gpu, shape, monkeypatch):
    """k_eval_bal at the edges of its schedule: E = NI = 1024 (every LDS table slot, two
    tables per point thread, 1023 free cameras on 256 work-groups x 4 slots), 300 cameras
    (4 waves per camera), 33 cameras (8 waves per camera, most work-groups without one) and
    a single free camera. Against the two-kernel pass: same iteration and CG counts, costs
    1e-10 relative; the fused pass must actually run (schedule 1)."""
    ncam, npt, opp = shape
    prob = pkg.synth(kind=0, num_cameras=ncam, num_points=npt, obs_per_point=opp, seed=60 + ncam)
    res, sched = [], []
    for fused in ("1", "0"):
        monkeypatch.setenv("DAB_EVAL_FUSED", fused)
        p = prob.copy()
        s = pkg.Solver(0)
        s.set_problem(p)
        sched.append(s.eval_fused())
        res.append(s.solve(pkg.options(max_num_iterations=6,
                                       linear_solver_type=pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)))
        s.close()
    assert sched == [1, 0]
    a, b = res
    assert [it["linear_solver_iterations"] for it in a["iterations"]] == \
        [it["linear_solver_iterations"] for it in b["iterations"]]
    for x, y in zip(a["iterations"], b["iterations"]):
        assert x["cost"] == pytest.approx(y["cost"], rel=1e-10 if x["success"] else 1e-8), (x, y)


def test_fused_camera_frame_small_angles(pkg, gpu, monkeypatch):
    """The fused pass accumulates the camera blocks in the point frame and applies J_l per
    camera afterwards; cameras on the small-angle tables (|w|^2 <= DBL_EPSILON, exactly
    zero or not) take X in place of R X there. Against the two-kernel pass (obs_rows, J_r
    per row) the LM trajectory must agree to 1e-10 relative (a 1.5e-8 Jacobian slip on
    those cameras would not)."""
    prob = pkg.synth(kind=0, num_cameras=60, num_points=6000, obs_per_point=8, seed=57)
    prob.ext[1, :3] = 0.0
    prob.ext[2, :3] = [1e-9, -2e-9, 3e-9]
    prob.ext[3, :3] = [0.0, 1.4e-8, 0.0]
    prob.ext[4, :3] = [1e-7, 0.0, 0.0]  # just above the threshold: the general tables
    res, sched = [], []
    for fused in ("1", "0"):
        monkeypatch.setenv("DAB_EVAL_FUSED", fused)
        p = prob.copy()
        s = pkg.Solver(0)
        s.set_problem(p)
        sched.append(s.eval_fused())
        res.append(s.solve(pkg.options(max_num_iterations=5)))
        s.close()
    assert sched == [1, 0]
    a, b = res
    assert [it["success"] for it in a["iterations"]] == [it["success"] for it in b["iterations"]]
    assert [it["linear_solver_iterations"] for it in a["iterations"]] == \
        [it["linear_solver_iterations"] for it in b["iterations"]]
    # accepted costs to 1e-10; the rejected candidates here are wild steps (costs ~1e23 from
    # ~1e7) whose cost amplifies the regrouped U, g_c rounding, so they get 1e-8
    for x, y in zip(a["iterations"], b["iterations"]):
        assert x["cost"] == pytest.approx(y["cost"], rel=1e-10 if x["success"] else 1e-8), (x, y)


@pytest.mark.parametrize("kind", ["bal", "c2"])
def test_split_fused_schedule_matches_single_launch(pkg, gpu, kind, monkeypatch):
    """The multi-rank schedule runs the fused kernel as a camera-side launch, then a
    point-side launch (the camera blocks' all-reduce overlaps the second). DAB_EVAL_SPLIT=1
    forces it on one rank, where both launches get the full grid: the LM trajectory must be
    bitwise that of the single fused launch (same wave split, fixed-point cost)."""
    if kind == "bal":
        prob = pkg.synth(kind=0, num_cameras=120, num_points=9000, obs_per_point=8, seed=54)
    else:
        prob = pkg.synth(**pkg.CONFIGS["c2_100cam"])
    monkeypatch.setenv("DAB_EVAL_FUSED", "1")
    res, pts, sched = [], [], []
    for split in ("0", "1"):
        monkeypatch.setenv("DAB_EVAL_SPLIT", split)
        p = prob.copy()
        s = pkg.Solver(0)
        s.set_problem(p)
        sched.append(s.eval_fused())
        res.append(s.solve(pkg.options(max_num_iterations=6,
                                       linear_solver_type=pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)))
        s.close()
        pts.append(p.points.copy())
    assert sched == [1, 2]
    assert [it["cost"] for it in res[0]["iterations"]] == [it["cost"] for it in res[1]["iterations"]]
    np.testing.assert_array_equal(pts[0], pts[1])


@pytest.mark.parametrize("wps", ["-112", "-122", "-113"])
@pytest.mark.parametrize("kind", ["bal", "rig"])
def test_prefetch_point_kernels_match(pkg, gpu, kind, wps, monkeypatch):
    """The prefetch-queue point kernels (DAB_EVAL_WPS <= -100: fixed-point cost, LDS
    intrinsics, single-extrinsic fast path for BAL) against the default LDS kernel in the
    two-kernel pass: same LM trajectory (cost 1e-10 relative)."""
    if kind == "bal":
        prob = pkg.synth(kind=0, num_cameras=50, num_points=5000, obs_per_point=7, seed=52)
    else:
        prob = pkg.synth(kind=1, num_arcs=5, num_rings=12, num_points=4000, obs_per_point=7, seed=53)
    monkeypatch.setenv("DAB_EVAL_FUSED", "0")
    res = []
    for w in ("-2", wps):
        monkeypatch.setenv("DAB_EVAL_WPS", w)
        p = prob.copy()
        s = pkg.Solver(0)
        s.set_problem(p)
        res.append(s.solve(pkg.options(max_num_iterations=10)))
        s.close()
    a, b = res
    assert len(a["iterations"]) == len(b["iterations"])
    np.testing.assert_allclose([it["cost"] for it in a["iterations"]], [it["cost"] for it in b["iterations"]],
                               rtol=1e-10)


def test_lm_freeze_camera_matches_oracle(pkg, orc, gpu):
    prob = pkg.synth(kind=1, num_arcs=4, num_rings=10, num_points=2000, obs_per_point=6, seed=23)
    prob.freeze_camera = True  # solve(..., freeze_camera=true), sfm.cc:111
    ext0 = prob.ext.copy()
    g, o, ref = run_both(pkg, orc, prob, max_num_iterations=20)
    assert_same_trajectory(g, o, prob, ref)
    np.testing.assert_array_equal(prob.ext, ext0)  # cameras untouched
    assert g["num_free_ext"] == 0


SMALL_SHAPES = {
    "one_point_two_cameras": dict(kind=0, num_cameras=2, num_points=1, obs_per_point=2, seed=71),
    "slice_63": dict(kind=0, num_cameras=3, num_points=63, obs_per_point=3, seed=72),
    "slice_64": dict(kind=0, num_cameras=3, num_points=64, obs_per_point=3, seed=73),
    "slice_65": dict(kind=0, num_cameras=3, num_points=65, obs_per_point=2, seed=74),
    "gauge_camera_only": dict(kind=0, num_cameras=1, num_points=7, obs_per_point=1, seed=75),
    "rig_one_arc_two_rings": dict(kind=1, num_arcs=1, num_rings=2, num_points=10, obs_per_point=2, seed=76),
    "rig_two_arcs_one_ring": dict(kind=1, num_arcs=2, num_rings=1, num_points=129, obs_per_point=2, seed=77),
}


@pytest.mark.parametrize("solver", ["explicit", "pcg"])
@pytest.mark.parametrize("shape", sorted(SMALL_SHAPES))
def test_small_shapes_match_oracle(pkg, orc, gpu, shape, solver):
    """Degenerate sizes against the oracle's trajectory: one point, SELL slices of 63/64/65
    points (a full slice, one short, one point over), no free camera (the only camera is the
    gauge: NC = 0), the smallest rigs. Costs that reach round-off (1e-15 .. 1e-20 on the
    noise-free shapes) are compared with an absolute floor of 1e-12 x the initial cost."""
    prob = pkg.synth(**SMALL_SHAPES[shape])
    lst = (pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR if solver == "explicit"
           else pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)
    g, o, ref = run_both(pkg, orc, prob, max_num_iterations=20, linear_solver_type=lst)
    floor = 1e-12 * o["initial_cost"]
    assert g["termination"] == o["termination"], (g["message"], o["message"])
    assert g["num_iterations"] == o["num_iterations"]
    assert g["initial_cost"] == pytest.approx(o["initial_cost"], rel=1e-12)
    for a, b in zip(g["iterations"], o["iterations"]):
        assert a["success"] == b["success"]
        assert abs(a["cost"] - b["cost"]) <= 1e-9 * abs(b["cost"]) + floor, (a, b)
    assert abs(g["final_cost"] - o["final_cost"]) <= 1e-9 * abs(o["final_cost"]) + floor
    assert np.abs(prob.points - ref.points).max() < 1e-7
    assert np.abs(prob.ext - ref.ext).max() < 1e-7


def test_gauge_and_unreferenced_blocks_untouched(pkg, orc, gpu):
    prob = pkg.synth(kind=0, num_cameras=20, num_points=600, obs_per_point=5, seed=24)
    # drop every observation of point 7 and of camera 3: those blocks leave the problem
    keep = (prob.obs_point != 7) & (prob.obs_ext0 != 3)
    sub = prob.subset(keep)
    sub.points = prob.points.copy()
    sub.ext = prob.ext.copy()
    before = (sub.points.copy(), sub.ext.copy())
    g, o, ref = run_both(pkg, orc, sub, max_num_iterations=15)
    assert_same_trajectory(g, o, sub, ref)
    np.testing.assert_array_equal(sub.points[7], before[0][7])
    np.testing.assert_array_equal(sub.ext[3], before[1][3])
    np.testing.assert_array_equal(sub.ext[0], before[1][0])  # gauge, sfm.cc:50-53


def test_observation_order_does_not_matter(pkg, gpu):
    prob = pkg.synth(kind=0, num_cameras=30, num_points=1500, obs_per_point=5, seed=25)
    perm = np.random.default_rng(0).permutation(prob.num_obs)
    shuffled = prob.subset(perm)
    shuffled.points, shuffled.ext = prob.points.copy(), prob.ext.copy()
    a, b = prob.copy(), shuffled
    opts = pkg.options(max_num_iterations=10)
    for p in (a, b):
        s = pkg.Solver(0)
        s.set_problem(p)
        s.solve(opts)
        s.close()
    # the library sorts by point (stable): identical per-point order -> bitwise identical
    # point results; camera sums follow entry order inside each point, also identical
    np.testing.assert_allclose(a.points, b.points, rtol=0, atol=1e-9)
    np.testing.assert_allclose(a.ext, b.ext, rtol=0, atol=1e-9)


def test_deterministic_bitwise(pkg, gpu):
    prob = pkg.synth(kind=1, num_arcs=5, num_rings=12, num_points=2500, obs_per_point=7, seed=26)
    outs = []
    for _ in range(2):
        p = prob.copy()
        s = pkg.Solver(0)
        s.set_problem(p)
        summ = s.solve(pkg.options(max_num_iterations=8))
        s.close()
        outs.append((p.points, p.ext, summ["final_cost"]))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])
    assert outs[0][2] == outs[1][2]


def test_empty_problem(pkg, gpu):
    prob = pkg.Problem(np.zeros((0, 2)), [], [], [], [], np.zeros((3, 3)), np.zeros((2, 6)),
                       np.array([[512, 512, 800, 800, 0, 0]], float), [1], [0])
    s = pkg.Solver(0)
    s.set_problem(prob)
    summ = s.solve(pkg.options())
    s.close()
    assert summ["termination"] == "CONVERGENCE" and summ["initial_cost"] == 0.0


def test_invalid_problem_rejected(pkg, gpu):
    prob = pkg.synth(kind=0, num_cameras=10, num_points=50, obs_per_point=3, seed=27)
    prob.obs_point[5] = 10 ** 6
    s = pkg.Solver(0)
    with pytest.raises(RuntimeError, match="out-of-range"):
        s.set_problem(prob)
    s.close()


def test_full_size_c3_properties(pkg, orc, gpu):
    """BASELINE config 3 (1k cams / 100k pts / 1M obs) at full size: size-independent
    properties (monotone accepted costs, gauge exact, Jacobian spot check vs oracle)."""
    prob = pkg.synth(**pkg.CONFIGS["c3_1kcam"])
    ext0 = prob.ext[0].copy()
    s = pkg.Solver(0)
    try:
        s.set_problem(prob)
        r, J = s.jacobians()
        idx = np.random.default_rng(1).choice(prob.num_obs, 2000, replace=False)
        sub = prob.subset(idx)
        ro, Jo = orc.eval_jacobians(pkg, sub)
        np.testing.assert_allclose(r[idx], ro, rtol=0, atol=1e-12 * np.abs(ro).max())
        scale = np.abs(Jo).reshape(len(Jo), -1).max(axis=1)
        assert (np.abs(J[idx] - Jo).reshape(len(Jo), -1).max(axis=1) / scale).max() < 1e-9
        summ = s.solve(pkg.options(max_num_iterations=6))
    finally:
        s.close()
    acc = [it["cost"] for it in summ["iterations"] if it["success"]]
    assert all(b < a for a, b in zip(acc, acc[1:]))
    assert summ["final_cost"] < 0.05 * summ["initial_cost"]
    np.testing.assert_array_equal(prob.ext[0], ext0)


@pytest.mark.parametrize("kind", ["bal", "rig"])
def test_schur_tiles_match_pair_tables(pkg, gpu, kind, monkeypatch):
    """EXPLICIT_SCHUR on small camera sets assembles S from fixed-point LDS tiles
    (k_schur_tiles, Y re-evaluated, integer sums); DAB_SCHUR_TILES=0 forces the camera-pair
    block sums over entry-pair tables. Same LM trajectory (cost 1e-10 relative, same
    iteration count and termination); the tile path is bitwise repeatable and the summary
    names the assembly that ran."""
    if kind == "bal":
        prob = pkg.synth(kind=0, num_cameras=70, num_points=5000, obs_per_point=8, seed=71)
    else:
        prob = pkg.synth(kind=1, num_arcs=6, num_rings=16, num_points=3000, obs_per_point=8, seed=72)
    res, pts = [], []
    for tiles in ("1", "0", "1"):
        monkeypatch.setenv("DAB_SCHUR_TILES", tiles)
        p = prob.copy()
        s = pkg.Solver(0)
        s.set_problem(p)
        res.append(s.solve(pkg.options(max_num_iterations=12)))
        s.close()
        pts.append(p.points.copy())
    a, b = res[0], res[1]
    assert a["schur_assembly"] == 1 and b["schur_assembly"] == 0
    assert a["linear_solver_type_used"] == pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR
    assert len(a["iterations"]) == len(b["iterations"]) and a["termination"] == b["termination"]
    np.testing.assert_allclose([it["cost"] for it in a["iterations"]], [it["cost"] for it in b["iterations"]],
                               rtol=1e-10)
    np.testing.assert_array_equal(pts[0], pts[2])


def test_schur_tiles_one_and_two_lds_buffers_agree(pkg, gpu, monkeypatch):
    """k_schur_tiles streams its batches through one LDS buffer (round 6's default: batches
    of up to 64 points) or two (DAB_TILE_SINGLE=0: half the records per batch, the next one
    in flight). The batches differ, so the blocks' partial sums are grouped differently: the
    same LM trajectory to rounding (cost 1e-12 relative, same iterations and termination)."""
    prob = pkg.synth(kind=1, num_arcs=8, num_rings=24, num_points=6000, obs_per_point=10, seed=74)
    res = []
    for single in ("1", "0"):
        monkeypatch.setenv("DAB_TILE_SINGLE", single)
        s = pkg.Solver(0)
        s.set_problem(prob.copy())
        res.append(s.solve(pkg.options(max_num_iterations=8)))
        s.close()
    a, b = res
    assert a["schur_assembly"] == 1 and b["schur_assembly"] == 1
    assert len(a["iterations"]) == len(b["iterations"]) and a["termination"] == b["termination"]
    np.testing.assert_allclose([it["cost"] for it in a["iterations"]], [it["cost"] for it in b["iterations"]],
                               rtol=1e-12)


@pytest.mark.parametrize("kind", ["bal", "rig"])
def test_large_initial_cost_matches_oracle(pkg, orc, gpu, kind):
    """A finite cost far beyond the old fixed-point range is an ordinary evaluation for
    Ceres: the solve proceeds. (1) The problem in pixel units scaled by 1e8 (focal lengths,
    principal points and observations; the same problem up to the residual scale, initial
    cost >= 1e20): the full trajectory must match the oracle's. (2) One observation 1e11 px
    off: the initial cost matches and the solve is not a FAILURE (its rejected candidates
    are too ill-conditioned to compare)."""
    if kind == "bal":
        prob = pkg.synth(kind=0, num_cameras=30, num_points=2000, obs_per_point=6, seed=73)
    else:
        prob = pkg.synth(kind=1, num_arcs=5, num_rings=10, num_points=2000, obs_per_point=6, seed=74)
    big = prob.copy()
    big.intr[:, :4] *= 1e8
    big.obs_xy *= 1e8
    g, o, ref = run_both(pkg, orc, big, max_num_iterations=10)
    assert g["initial_cost"] >= 1e20
    assert_same_trajectory(g, o, big, ref)
    out = prob.copy()
    out.obs_xy[17] = [1.0e11, -3.0e10]
    g, o, ref = run_both(pkg, orc, out, max_num_iterations=10)
    assert g["initial_cost"] >= 1e20
    assert g["initial_cost"] == pytest.approx(o["initial_cost"], rel=1e-12)
    assert g["termination"] != "FAILURE", g["message"]
    assert [it["success"] for it in g["iterations"]] == [it["success"] for it in o["iterations"]]


@pytest.mark.parametrize("kind", ["bal", "rig"])
def test_noise_free_problem_matches_oracle(pkg, orc, gpu, kind):
    """Observations without pixel noise: the cost falls towards zero, where a coarse
    fixed-point cost would quantise the function-tolerance and relative-decrease tests.
    The cost accumulator holds partials exactly down to 2^-100, so the GPU's iterations
    match the oracle's while the cost is above 1e-12 of the initial one (below that both
    are rounding noise), both converge, and the parameters agree to 1e-9."""
    if kind == "bal":
        prob = pkg.synth(kind=0, num_cameras=30, num_points=2000, obs_per_point=6, seed=81, pixel_noise=0.0)
    else:
        prob = pkg.synth(kind=1, num_arcs=5, num_rings=10, num_points=2000, obs_per_point=6, seed=82,
                         pixel_noise=0.0)
    g, o, ref = run_both(pkg, orc, prob, max_num_iterations=30)
    c0 = o["initial_cost"]
    assert g["initial_cost"] == pytest.approx(c0, rel=1e-12)
    for a, b in zip(g["iterations"], o["iterations"]):
        if b["cost"] < 1e-12 * c0:
            break
        assert a["success"] == b["success"]
        assert a["cost"] == pytest.approx(b["cost"], rel=1e-6), (a["cost"], b["cost"])
    assert g["termination"] == "CONVERGENCE" and o["termination"] == "CONVERGENCE"
    assert g["final_cost"] < 1e-12 * c0 and o["final_cost"] < 1e-12 * c0
    np.testing.assert_allclose(prob.points, ref.points, rtol=0, atol=1e-9)


@pytest.mark.parametrize("knob", ["DAB_CHOL_BACK_FLOW=0", "DAB_CHOL_FUSE_PANEL=0", "DAB_CHOL_PREFACTOR=0",
                                  "DAB_CHOL_V1=1", "DAB_CHOL_GROUP=3", "DAB_CHOL_GRAPH_MIN=1",
                                  "DAB_CHOL_STRIP=0", "DAB_CHOL_STRIP=0,DAB_CHOL_GRAPH_MIN=1",
                                  "DAB_CHOL_GROUP=3,DAB_CHOL_GRAPH_MIN=1"])
def test_cholesky_schedules_agree(pkg, gpu, knob, monkeypatch):
    """The dense Cholesky's schedules — the dataflow back substitution against the
    grid-barrier one, the panel step fused into the column update against its own launch,
    the diagonal block factored by the column update against every panel work-group, and
    the round-1 per-step schedule, bulk updates over panel triples instead of pairs, the
    round-5 strip schedule (the bulk's first block column a launch of its own) against the
    single bulk launch, and the captured graph against direct launches (13 blocks launch
    directly by default) — solve
    the same systems: the EXPLICIT LM trajectories agree to 1e-10 relative. n = 6 x 130 =
    780 (13 blocks, a short last block)."""
    prob = pkg.synth(kind=0, num_cameras=130, num_points=6000, obs_per_point=8, seed=57)
    opts = pkg.options(max_num_iterations=6, linear_solver_type=pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR)
    kv = [a.split("=") for a in knob.split(",")]
    res = []
    for on in (False, True):
        for name, val in kv:
            if on:
                monkeypatch.setenv(name, val)
            else:
                monkeypatch.delenv(name, raising=False)
        s = pkg.Solver(0)
        try:
            s.set_problem(prob.copy())
            res.append(s.solve(opts))
        finally:
            s.close()
    a, b = res
    assert a["num_iterations"] == b["num_iterations"] and a["termination"] == b["termination"]
    np.testing.assert_allclose([it["cost"] for it in a["iterations"]], [it["cost"] for it in b["iterations"]],
                               rtol=1e-10)
