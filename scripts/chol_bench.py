"""Time the device dense Cholesky + solves on an n x n SPD system (default n = 6000, the
reduced camera system of BASELINE config 3) and check it against numpy."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkgload  # noqa: E402

pkg = _pkgload.load()
if os.environ.get("DAB_LIB"):  # another build of libdab (A/B)
    abi = sys.modules[pkg.__name__ + "._abi"]
    abi._LIB = abi.load_library(os.path.join(ROOT, os.environ["DAB_LIB"]))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 6000
rng = np.random.default_rng(0)
M = rng.standard_normal((n, n)) / np.sqrt(n)
A = M @ M.T + np.eye(n)
b = rng.standard_normal(n)
s = pkg.Solver(0)
times = []
for it in range(6):
    x, ms, ok = s.dense_spd_solve(A, b)
    times.append(ms)
s.close()
t0 = time.perf_counter()
ref = np.linalg.solve(A, b)
t_np = time.perf_counter() - t0
err = np.linalg.norm(x - ref) / np.linalg.norm(ref)
if os.environ.get("DAB_DUMP"):  # the solution, for a bitwise A/B of two builds
    np.save(os.environ["DAB_DUMP"], x)
gflop = n ** 3 / 3 / 1e9
print(f"n={n} ok={ok} device ms: first {times[0]:.3f} median {np.median(times[1:]):.3f} "
      f"({gflop / (np.median(times[1:]) * 1e-3) / 1e3:.2f} TFLOP/s on n^3/3); "
      f"rel err vs numpy {err:.2e}; numpy (host LAPACK) {t_np * 1e3:.1f} ms")
