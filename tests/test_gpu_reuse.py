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


def test_solve_continues_on_same_problem(pkg, gpu):
    """Two solves of 3 iterations on one handle and problem (the second starts from the
    first's result, as sfm.cc's repeated solve() calls) against one fresh solve each: the
    second solve of the reused handle equals a fresh handle started from the same
    parameters, for the exact step (sticky dense S, captured Cholesky graph) and PCG."""
    prob = pkg.synth(kind=0, num_cameras=60, num_points=3000, obs_per_point=6, seed=87)
    for lst in (pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR, pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG,
                pkg.DAB_LINEAR_SOLVER_AUTO):
        p = prob.copy()
        s = pkg.Solver(0)
        try:
            s.set_problem(p)
            s.solve(pkg.options(max_num_iterations=3, linear_solver_type=lst))
            mid_pts, mid_ext = p.points.copy(), p.ext.copy()
            s.set_problem(p)  # the re-set of the same shape keeps S and the graph
            b = s.solve(pkg.options(max_num_iterations=3, linear_solver_type=lst))
        finally:
            s.close()
        q = prob.copy()
        q.points[:] = mid_pts
        q.ext[:] = mid_ext
        f = pkg.Solver(0)
        try:
            f.set_problem(q)
            c = f.solve(pkg.options(max_num_iterations=3, linear_solver_type=lst))
        finally:
            f.close()
        assert [it["cost"] for it in b["iterations"]] == [it["cost"] for it in c["iterations"]]
        np.testing.assert_array_equal(p.points, q.points)
        np.testing.assert_array_equal(p.ext, q.ext)
        if lst == pkg.DAB_LINEAR_SOLVER_AUTO:  # one rank: AUTO is the exact step
            assert b["linear_solver_type_used"] == pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR


def test_filter_then_resolve_matches_fresh(pkg, gpu):
    """dab_filter on the solve's resident problem, then the caller drops the filtered
    observations and re-sets the same handle (the sfm.cc loop): same trajectory as a
    fresh handle on the filtered problem."""
    prob = pkg.synth(kind=1, num_arcs=5, num_rings=14, num_points=4000, obs_per_point=7, seed=88)
    lst = pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR
    s = pkg.Solver(0)
    try:
        p = prob.copy()
        s.set_problem(p)
        s.solve(pkg.options(max_num_iterations=3, linear_solver_type=lst))
        for bound in (4.0, 2.0, 1.0, 0.5, 0.25, 0.1):  # a boundary that drops some
            obs_keep, _ = s.filter(bound, [0.0, 0.0, 0.0], 1e9)
            keep = np.nonzero(np.asarray(obs_keep))[0]
            if 0 < len(keep) < p.num_obs:
                break
        assert 0 < len(keep) < p.num_obs
        q = p.subset(keep)
        q_fresh = q.copy()
        s.set_problem(q)
        a = s.solve(pkg.options(max_num_iterations=3, linear_solver_type=lst))
    finally:
        s.close()
    f = pkg.Solver(0)
    try:
        f.set_problem(q_fresh)
        b = f.solve(pkg.options(max_num_iterations=3, linear_solver_type=lst))
    finally:
        f.close()
    assert [it["cost"] for it in a["iterations"]] == [it["cost"] for it in b["iterations"]]
    np.testing.assert_array_equal(q.points, q_fresh.points)


def test_release_caches_between_handles(pkg, gpu):
    """dab_release_caches (round 5): with one handle alive and after it is destroyed, the
    cached streams and pinned blocks are dropped; handles created afterwards take fresh ones
    and give bitwise the same trajectory."""
    prob = pkg.synth(kind=0, num_cameras=20, num_points=1500, obs_per_point=6, seed=85)
    lib = pkg.load_library()
    ex = pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR
    s = pkg.Solver(0)
    try:
        ref = _solve(pkg, s, prob, ex)
        assert lib.dab_release_caches() == 0  # a live handle keeps its own streams
        again = _solve(pkg, s, prob, ex)
    finally:
        s.close()
    assert lib.dab_release_caches() == 0
    assert lib.dab_release_caches() == 0  # idempotent
    s = pkg.Solver(0)
    try:
        got = _solve(pkg, s, prob, ex)
    finally:
        s.close()
    for other in (again, got):
        assert other[0] == ref[0]
        np.testing.assert_array_equal(other[2], ref[2])
        np.testing.assert_array_equal(other[3], ref[3])
