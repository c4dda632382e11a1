"""The device dense Cholesky (reduced camera system of the DENSE_SCHUR-equivalent solver)
against numpy/LAPACK on random SPD systems. Tolerance: relative residual and relative
error vs numpy.linalg.solve <= 1e-12 * cond-scaled bound (well-conditioned inputs)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 6, 63, 64, 65, 127, 128, 130, 191, 192, 193, 256, 257, 384, 449, 1000, 2048, 2050, 3001])
def test_dense_spd_solve_matches_numpy(pkg, gpu, n):
    check_solve(pkg, n)


def check_solve(pkg, n):
    rng = np.random.default_rng(n)
    M = rng.standard_normal((n, n))
    A = M @ M.T + n * np.eye(n)
    b = rng.standard_normal(n)
    s = pkg.Solver(0)
    try:
        x, ms, ok = s.dense_spd_solve(np.tril(A) + np.triu(rng.standard_normal((n, n)), 1), b)
    finally:
        s.close()
    assert ok
    ref = np.linalg.solve(A, b)
    assert np.linalg.norm(x - ref) <= 1e-12 * np.linalg.cond(A) * np.linalg.norm(ref)
    assert np.linalg.norm(A @ x - b) <= 1e-12 * np.linalg.norm(A) * np.linalg.norm(x)


def test_dense_spd_solve_detects_indefinite(pkg, gpu):
    n = 100
    A = np.eye(n)
    A[57, 57] = -1.0
    s = pkg.Solver(0)
    try:
        _, _, ok = s.dense_spd_solve(A, np.ones(n))
    finally:
        s.close()
    assert not ok
