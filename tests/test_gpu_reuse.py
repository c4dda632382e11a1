"""One handle across problems of different shapes (the host adapter keeps one libdab handle
for a whole sfm.cc pipeline): solving problem B after problem A on the same handle must give
bitwise the trajectory of a fresh handle on B. Covers the round-2 advisor finding that a
matrix-free rig solve left the CG update pointed at its freed work-group partials, and two
found by these tests: the single-pass product's grid size outlived its problem (a small rig
followed by a large-camera rig ran the single-pass product on freed partials, results off
in the last bits), and the lazily allocated fp32 Y records kept a freed pointer."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _solve(pkg, s, prob, lst, iters=4, **kw):
    p = prob.copy()
    s.set_problem(p)
    summ = s.solve(pkg.options(max_num_iterations=iters, linear_solver_type=lst, **kw))
    return [it["cost"] for it in summ["iterations"]], \
        [it["linear_solver_iterations"] for it in summ["iterations"]], p.points.copy(), p.ext.copy()


def test_handle_reuse_small_rig_then_large_rig(pkg, gpu):
    small = pkg.synth(kind=1, num_arcs=4, num_rings=10, num_points=1500, obs_per_point=6, seed=81)
    large = pkg.synth(kind=1, num_arcs=12, num_rings=160, num_points=6000, obs_per_point=8, seed=82)
    assert large.ext.shape[0] > 161  # more than 160 free cameras: stored-Y PCG with cross blocks
    pcg = pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG
    fresh = pkg.Solver(0)
    try:
        ref = _solve(pkg, fresh, large, pcg)
    finally:
        fresh.close()
    s = pkg.Solver(0)
    try:
        _solve(pkg, s, small, pcg)                                   # matrix-free product
        _solve(pkg, s, small, pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR)  # block tiles + Cholesky
        got = _solve(pkg, s, large, pcg)
    finally:
        s.close()
    assert got[0] == ref[0]
    assert got[1] == ref[1]
    np.testing.assert_array_equal(got[2], ref[2])
    np.testing.assert_array_equal(got[3], ref[3])


def test_handle_reuse_large_then_small(pkg, gpu):
    """The other order, and the exact step after PCG on the same handle."""
    small = pkg.synth(kind=1, num_arcs=4, num_rings=10, num_points=1500, obs_per_point=6, seed=83)
    large = pkg.synth(kind=0, num_cameras=200, num_points=4000, obs_per_point=6, seed=84)
    fresh = pkg.Solver(0)
    try:
        ref_e = _solve(pkg, fresh, small, pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR)
        ref_p = _solve(pkg, fresh, small, pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)
    finally:
        fresh.close()
    s = pkg.Solver(0)
    try:
        _solve(pkg, s, large, pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR)      # pair tables
        _solve(pkg, s, large, pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)  # stored-Y PCG
        got_e = _solve(pkg, s, small, pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR)
        got_p = _solve(pkg, s, small, pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)
    finally:
        s.close()
    for got, ref in ((got_e, ref_e), (got_p, ref_p)):
        assert got[0] == ref[0]
        assert got[1] == ref[1]
        np.testing.assert_array_equal(got[2], ref[2])
        np.testing.assert_array_equal(got[3], ref[3])


def test_handle_reuse_fp32_stored_y(pkg, gpu):
    """Mixed-precision stored-Y PCG (fp32 Y records, allocated on first use) on a handle
    that already ran it on another problem: the records are allocated again, not reused
    from the freed set."""
    a = pkg.synth(kind=0, num_cameras=220, num_points=5000, obs_per_point=6, seed=85)
    b = pkg.synth(kind=0, num_cameras=240, num_points=7000, obs_per_point=7, seed=86)
    pcg = pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG
    fresh = pkg.Solver(0)
    try:
        ref = _solve(pkg, fresh, b, pcg, pcg_fp32=1)
    finally:
        fresh.close()
    s = pkg.Solver(0)
    try:
        _solve(pkg, s, a, pcg, pcg_fp32=1)
        got = _solve(pkg, s, b, pcg, pcg_fp32=1)
    finally:
        s.close()
    assert got[0] == ref[0]
    assert got[1] == ref[1]
    np.testing.assert_array_equal(got[2], ref[2])
