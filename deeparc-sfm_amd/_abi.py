"""ctypes mirror of include/dab.h (the C ABI of libdab.so).

Only plain structs and the shared-library loader live here. The library is built
in-tree (deeparc-sfm_amd/libdab.so, ``make -C deeparc-sfm_amd``); there is no CPU
fallback — loading fails loudly if the HIP build is missing.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libdab.so")

DAB_OK = 0
DAB_LINEAR_SOLVER_EXPLICIT_SCHUR = 0
DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG = 1
DAB_LINEAR_SOLVER_AUTO = 2
DAB_CONVERGENCE = 0
DAB_NO_CONVERGENCE = 1
DAB_FAILURE = 2
TERMINATION = {0: "CONVERGENCE", 1: "NO_CONVERGENCE", 2: "FAILURE"}

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)
_u8p = C.POINTER(C.c_uint8)


class DabProblem(C.Structure):
    _fields_ = [
        ("num_obs", C.c_int32), ("num_points", C.c_int32), ("num_ext", C.c_int32),
        ("num_intr", C.c_int32),
        ("obs_xy", _dp), ("obs_point", _ip), ("obs_ext0", _ip), ("obs_ext1", _ip),
        ("obs_intr", _ip), ("points", _dp), ("ext", _dp), ("intr", _dp),
        ("intr_nf", _ip), ("intr_nk", _ip), ("ext_const", _u8p),
        ("freeze_camera", C.c_int32), ("reserved", C.c_int32),
    ]


class DabOptions(C.Structure):
    _fields_ = [
        ("max_num_iterations", C.c_int32), ("linear_solver_type", C.c_int32),
        ("max_solver_time_in_seconds", C.c_double), ("function_tolerance", C.c_double),
        ("gradient_tolerance", C.c_double), ("parameter_tolerance", C.c_double),
        ("min_relative_decrease", C.c_double), ("initial_trust_region_radius", C.c_double),
        ("max_trust_region_radius", C.c_double), ("min_trust_region_radius", C.c_double),
        ("min_lm_diagonal", C.c_double), ("max_lm_diagonal", C.c_double),
        ("max_num_consecutive_invalid_steps", C.c_int32), ("jacobi_scaling", C.c_int32),
        ("minimizer_progress_to_stdout", C.c_int32), ("num_threads", C.c_int32),
        ("max_linear_solver_iterations", C.c_int32), ("min_linear_solver_iterations", C.c_int32),
        ("eta", C.c_double), ("pcg_fp32", C.c_int32), ("reserved", C.c_int32),
    ]


class DabIteration(C.Structure):
    _fields_ = [
        ("iteration", C.c_int32), ("step_is_successful", C.c_int32),
        ("step_is_valid", C.c_int32), ("linear_solver_iterations", C.c_int32),
        ("cost", C.c_double), ("cost_change", C.c_double), ("gradient_max_norm", C.c_double),
        ("step_norm", C.c_double), ("relative_decrease", C.c_double),
        ("trust_region_radius", C.c_double), ("iteration_time_in_seconds", C.c_double),
    ]


class DabSummary(C.Structure):
    _fields_ = [
        ("initial_cost", C.c_double), ("final_cost", C.c_double),
        ("num_iterations", C.c_int32), ("num_successful_steps", C.c_int32),
        ("num_unsuccessful_steps", C.c_int32), ("termination_type", C.c_int32),
        ("num_residuals", C.c_int32), ("num_parameters", C.c_int32),
        ("num_free_points", C.c_int32), ("num_free_ext", C.c_int32),
        ("total_time_in_seconds", C.c_double),
        ("jacobian_evaluation_time_in_seconds", C.c_double),
        ("residual_evaluation_time_in_seconds", C.c_double),
        ("linear_solver_time_in_seconds", C.c_double),
        ("message", C.c_char * 256),
        ("iterations", C.POINTER(DabIteration)), ("iterations_capacity", C.c_int32),
        ("iterations_written", C.c_int32), ("linear_solver_type_used", C.c_int32),
        ("schur_assembly", C.c_int32),
    ]


class DabSynthConfig(C.Structure):
    _fields_ = [
        ("kind", C.c_int32), ("num_cameras", C.c_int32), ("num_arcs", C.c_int32),
        ("num_rings", C.c_int32), ("num_points", C.c_int32), ("obs_per_point", C.c_int32),
        ("seed", C.c_uint64), ("point_seed", C.c_uint64), ("pixel_noise", C.c_double),
        ("point_noise", C.c_double),
        ("rot_noise", C.c_double), ("trans_noise", C.c_double),
    ]


# int (*)(double* buf, int64_t count, int op, void* user): op 0 = sum, 1 = max
HostAllreduceFn = C.CFUNCTYPE(C.c_int, _dp, C.c_int64, C.c_int, C.c_void_p)

# name -> (restype, argtypes); every symbol include/dab.h declares
SIGNATURES = {
    "dab_abi_version": (C.c_int, []),
    "dab_last_error": (C.c_char_p, []),
    "dab_options_init": (None, [C.POINTER(DabOptions)]),
    "dab_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "dab_comm_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
    "dab_create_dist": (C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint8),
                                  C.POINTER(C.c_void_p)]),
    "dab_create_dist_host": (C.c_int, [C.c_int, C.c_int, C.c_int, HostAllreduceFn, C.c_void_p,
                                       C.POINTER(C.c_void_p)]),
    "dab_destroy": (C.c_int, [C.c_void_p]),
    "dab_release_caches": (C.c_int, []),
    "dab_set_problem": (C.c_int, [C.c_void_p, C.POINTER(DabProblem)]),
    "dab_update_parameters": (C.c_int, [C.c_void_p, _dp, _dp]),
    "dab_solve": (C.c_int, [C.c_void_p, C.POINTER(DabOptions), C.POINTER(DabSummary)]),
    "dab_get_parameters": (C.c_int, [C.c_void_p, _dp, _dp]),
    "dab_eval_residuals": (C.c_int, [C.c_void_p, _dp, _dp]),
    "dab_eval_jacobians": (C.c_int, [C.c_void_p, _dp, _dp]),
    "dab_filter": (C.c_int, [C.c_void_p, C.c_double, _dp, C.c_double, _u8p, _u8p, _ip, _ip]),
    "dab_dense_spd_solve": (C.c_int, [C.c_void_p, C.c_int, _dp, _dp, _dp, _dp]),
    "dab_bench_eval_pass": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "dab_sync": (C.c_int, [C.c_void_p]),
    "dab_bench_kernel_ms": (C.c_int, [C.c_void_p, _dp, _dp]),
    "dab_jacobian_bytes": (C.c_int, [C.c_void_p, _dp]),
    "dab_bench_pair_ms": (C.c_int, [C.c_void_p, _dp, _dp]),
    "dab_eval_schedule": (C.c_int, [C.c_void_p, _ip]),
    "dab_pcg_schedule": (C.c_int, [C.c_void_p, _ip]),
    "dab_comm_schedule": (C.c_int, [C.c_void_p, _ip]),
    "dab_synth_sizes": (C.c_int, [C.POINTER(DabSynthConfig), _ip, _ip, _ip, _ip]),
    "dab_synth_fill": (C.c_int, [C.POINTER(DabSynthConfig), C.POINTER(DabProblem), _u8p]),
}

_LIB = None


def load_library(path=None):
    """Load libdab.so (the HIP build). Raises if it is missing: there is no fallback."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(
            f"libdab.so not found at {p}: build it with `make -C deeparc-sfm_amd` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = C.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.dab_abi_version() != 2:
        raise RuntimeError("libdab ABI version mismatch")
    if path is None:
        _LIB = lib
    return lib


def last_error(lib=None):
    lib = lib or load_library()
    msg = lib.dab_last_error()
    return msg.decode() if msg else ""


def check(rc, lib=None):
    if rc != 0:
        raise RuntimeError(f"libdab error {rc}: {last_error(lib)}")
    return rc
