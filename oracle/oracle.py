"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of the CPU oracle (oracle/liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this, as the
checker. The product (libdab.so) never links or calls it. See dab_oracle.c's header for
what it restates and its parity status (pinned to tests/golden/ fixtures; against Ceres
itself: parity unpinned — Ceres cannot be built here).
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib(abi):
    """abi: the deeparc_sfm_amd._abi module (struct definitions shared with the product)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
        L.orc_eval_residuals.argtypes = [C.POINTER(abi.DabProblem), dp, dp]
        L.orc_eval_jacobians.argtypes = [C.POINTER(abi.DabProblem), dp, dp, C.c_int]
        L.orc_solve.argtypes = [C.POINTER(abi.DabProblem), C.POINTER(abi.DabOptions),
                                C.POINTER(abi.DabSummary)]
        L.orc_angle_axis_rotate_point.argtypes = [dp, dp, dp]
        L.orc_angle_axis_to_rotation_matrix.argtypes = [dp, dp]
        L.orc_quaternion_to_angle_axis.argtypes = [dp, dp]
        L.orc_rotation_matrix_to_angle_axis.argtypes = [dp, dp]
        _lib = L
    return _lib


def _d(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def eval_jacobians(pkg, problem, num_threads=0):
    L = lib(pkg._abi)
    n = problem.num_obs
    r = np.zeros((n, 2))
    J = np.zeros((n, 2, 15))
    cp = problem.as_c()
    L.orc_eval_jacobians(C.byref(cp), _d(r), _d(J), num_threads)
    return r, J


def eval_residuals(pkg, problem):
    L = lib(pkg._abi)
    r = np.zeros((problem.num_obs, 2))
    cost = C.c_double()
    cp = problem.as_c()
    L.orc_eval_residuals(C.byref(cp), _d(r), C.byref(cost))
    return r, cost.value


def solve(pkg, problem, opts, max_records=1024):
    """Runs the CPU LM (DENSE_SCHUR restatement) in place on problem.points/ext."""
    L = lib(pkg._abi)
    its = (pkg._abi.DabIteration * max_records)()
    s = pkg._abi.DabSummary()
    s.iterations = C.cast(its, C.POINTER(pkg._abi.DabIteration))
    s.iterations_capacity = max_records
    cp = problem.as_c()
    L.orc_solve(C.byref(cp), C.byref(opts), C.byref(s))
    return pkg.core.summary_to_dict(s, its)


def rotate_point(aa, pt):
    L = lib(_abi_stub())
    out = np.zeros(3)
    L.orc_angle_axis_rotate_point(_d(np.ascontiguousarray(aa, float)),
                                  _d(np.ascontiguousarray(pt, float)), _d(out))
    return out


def aa_to_rotmat(aa):
    L = lib(_abi_stub())
    out = np.zeros(9)
    L.orc_angle_axis_to_rotation_matrix(_d(np.ascontiguousarray(aa, float)), _d(out))
    return out


def quat_to_aa(q):
    L = lib(_abi_stub())
    out = np.zeros(3)
    L.orc_quaternion_to_angle_axis(_d(np.ascontiguousarray(q, float)), _d(out))
    return out


def rotmat_to_aa(R):
    L = lib(_abi_stub())
    out = np.zeros(3)
    L.orc_rotation_matrix_to_angle_axis(_d(np.ascontiguousarray(R, float)), _d(out))
    return out


def _abi_stub():
    import sys
    mod = sys.modules.get("deeparc_sfm_amd")
    if mod is None:
        import importlib
        root = os.path.dirname(HERE)
        import sys as _s
        _s.path.insert(0, root)
        mod = importlib.import_module("_pkgload").load()
    return mod._abi
