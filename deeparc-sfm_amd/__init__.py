"""deeparc-sfm_amd — MI355X-native bundle-adjustment hot path for pureexe/deeparc-sfm.

The product is libdab.so (gfx950 HIP kernels + C ABI, include/dab.h) plus the C++ host
adapter; this Python package is a thin ctypes mirror used by tests and bench.py.
Import it as ``deeparc_sfm_amd`` via _pkgload.load() (the directory name has a hyphen).
"""
from ._abi import (DAB_CONVERGENCE, DAB_FAILURE, DAB_LINEAR_SOLVER_AUTO, DAB_LINEAR_SOLVER_EXPLICIT_SCHUR,
                   DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG, DAB_NO_CONVERGENCE, LIB_PATH,
                   SIGNATURES, load_library, last_error)
from .core import CONFIGS, Problem, Solver, options, solve, synth, synth_config

__all__ = [
    "CONFIGS", "Problem", "Solver", "options", "solve", "synth", "synth_config",
    "load_library", "last_error", "LIB_PATH", "SIGNATURES",
    "DAB_CONVERGENCE", "DAB_NO_CONVERGENCE", "DAB_FAILURE",
    "DAB_LINEAR_SOLVER_EXPLICIT_SCHUR", "DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG", "DAB_LINEAR_SOLVER_AUTO",
]
