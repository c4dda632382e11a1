"""The CPU oracle (checker) pinned against the independent golden vectors.

Golden vectors: tests/golden/*.json from oracle/gen_golden.py (sympy symbolic derivative of
the SnavelyReprojectionError functor, snavely_reprojection_error.hh:39-118, with Ceres'
rotation branch semantics, evaluated at 40 digits). Against Ceres itself parity is
unpinned: the reference cannot be built here."""
import numpy as np
import pytest

from golden_util import (TOL_JAC, TOL_JAC_AUTODIFF_NEAR, TOL_RES, cases_problem, functor_cases,
                         golden_arrays, rotation_cases)


def test_golden_coverage():
    cases = functor_cases()
    assert len(cases) >= 100
    combos = {(c["nf"], c["nk"], c["compose"], c["regime"]) for c in cases}
    assert len(combos) == 2 * 3 * 2 * 4  # |f| x |k| x {single, arc∘ring} x branch regimes


def test_oracle_residual_and_autodiff_jacobian(pkg, orc):
    cases = functor_cases()
    p = cases_problem(pkg, cases)
    r, J = orc.eval_jacobians(pkg, p)
    rg, Jg = golden_arrays(cases)
    for i, c in enumerate(cases):
        er = np.abs(r[i] - rg[i]).max() / max(1.0, np.abs(rg[i]).max())
        assert er < TOL_RES, (i, c["regime"], er)
        eJ = np.abs(J[i] - Jg[i]).max() / np.abs(Jg[i]).max()
        tol = TOL_JAC_AUTODIFF_NEAR if c["regime"] == "near" else TOL_JAC
        assert eJ < tol, (i, c["regime"], c["compose"], eJ)


def test_oracle_residual_only_pass_matches_jet_pass(pkg, orc):
    cases = functor_cases()
    p = cases_problem(pkg, cases)
    r1, _ = orc.eval_jacobians(pkg, p)
    r2, cost = orc.eval_residuals(pkg, p)
    # ceres::Jet division computes f.a * (1/g.a) where T=double computes f/g, so the two
    # passes agree to a few ulps, not bitwise (the same holds inside Ceres)
    np.testing.assert_allclose(r1, r2, rtol=1e-14, atol=1e-12)
    assert cost == pytest.approx(0.5 * (r2 ** 2).sum(), rel=1e-15)


def test_rotation_helpers(orc):
    for c in rotation_cases():
        out = orc.rotate_point(c["aa"], c["point"])
        np.testing.assert_allclose(out, c["rotated"], rtol=0, atol=2e-15)
        th = np.linalg.norm(c["aa"])
        if th > 1e-6:  # the conversions are exact only away from the identity
            np.testing.assert_allclose(orc.quat_to_aa(c["quat"]), c["aa"], rtol=0, atol=1e-14)
            np.testing.assert_allclose(orc.rotmat_to_aa(c["R_colmajor"]), c["aa"], rtol=0, atol=1e-13)
        R = orc.aa_to_rotmat(c["aa"])
        if th * th > 2.220446049250313e-16:
            np.testing.assert_allclose(R, c["R_colmajor"], rtol=0, atol=1e-15)


def test_oracle_pcg_reaches_dense_schur_minimum(pkg, orc):
    """The oracle's CG step (implicit-Schur PCG restatement) converges to the same
    minimum as its exact dense-Schur step on a small rig problem."""
    prob = pkg.synth(kind=1, num_arcs=4, num_rings=8, num_points=400, obs_per_point=6, seed=41)
    out = {}
    for name, lst in (("dense", pkg.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR),
                      ("pcg", pkg.DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG)):
        p = prob.copy()
        out[name] = orc.solve(pkg, p, pkg.options(max_num_iterations=40, num_threads=4,
                                                  linear_solver_type=lst))
    assert out["pcg"]["final_cost"] == pytest.approx(out["dense"]["final_cost"], rel=1e-4)
    assert out["pcg"]["final_cost"] < 0.05 * out["pcg"]["initial_cost"]
    cg = [it["linear_solver_iterations"] for it in out["pcg"]["iterations"][1:]]
    assert max(cg) > 1 and all(c <= 500 for c in cg)
