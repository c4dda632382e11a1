"""ctypes binding of the host adapter (include/deeparc_host.h, libdeeparc_host.so).

The C++ adapter mirrors the reference's DeepArcManager (src/DeepArcManager.hh) and the
sfm.cc driver functions over libdab. This module exposes the same names to Python:
    m = DeepArcManager(); m.read(path); solve(m, 100, 3600, freeze_camera=True)
    m.filterPoint3d(5.0, center, radius); m.write(path); m.writePly(path)
    center, radius = fit_hemisphere(m.getCameraCenter())
The library raises RuntimeError when the reference would throw.
"""
import ctypes as C
import os

import numpy as np

from . import _abi

HOST_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libdeeparc_host.so")
_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)

# dam_pipeline_report's breakdown fields, in order
PIPELINE_STAGES = ("read", "fit", "write", "marshal", "setup", "update", "prep", "lm", "writeback", "filter_device",
                   "filter_host")


class PipelineReport(C.Structure):  # dam_pipeline_report
    _fields_ = [("hemisphere_center", C.c_double * 3), ("hemisphere_radius", C.c_double),
                ("rounds", C.c_int32), ("final_blocks", C.c_int32), ("final_points", C.c_int32),
                ("solves", C.c_int32), ("lm_iterations", C.c_int32), ("reserved", C.c_int32),
                ("final_cost", C.c_double), ("solve_seconds", C.c_double), ("filter_seconds", C.c_double),
                ("total_seconds", C.c_double)] + [(k + "_seconds", C.c_double) for k in PIPELINE_STAGES]


SIGNATURES = {
    "dam_last_error": (C.c_char_p, []),
    "dam_create": (C.c_int, [C.POINTER(C.c_void_p)]),
    "dam_destroy": (C.c_int, [C.c_void_p]),
    "dam_read": (C.c_int, [C.c_void_p, C.c_char_p]),
    "dam_write": (C.c_int, [C.c_void_p, C.c_char_p]),
    "dam_write_ply": (C.c_int, [C.c_void_p, C.c_char_p]),
    "dam_sizes": (C.c_int, [C.c_void_p, _ip, _ip, _ip, _ip, _ip, _ip, _ip]),
    "dam_get_points": (C.c_int, [C.c_void_p, _dp, _ip]),
    "dam_get_cameras": (C.c_int, [C.c_void_p, _dp, _dp]),
    "dam_get_blocks": (C.c_int, [C.c_void_p, _ip, _ip, _ip, _dp]),
    "dam_solve": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                            C.POINTER(_abi.DabSummary)]),
    "dam_filter": (C.c_int, [C.c_void_p, C.c_double, _dp, C.c_double]),
    "dam_camera_centers": (C.c_int, [C.c_void_p, _dp, C.c_int32, _ip]),
    "dam_fit_hemisphere": (C.c_int, [_dp, C.c_int32, _dp, _dp, C.c_int32]),
    "dam_run_pipeline": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int32, C.c_int32, C.c_double,
                                   _dp, _ip]),
    "dam_run_pipeline_report": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int32, C.c_int32, C.c_double,
                                          C.c_int32, C.POINTER(PipelineReport)]),
}

_LIB = None


def load_host_library():
    global _LIB
    if _LIB is None:
        _abi.load_library()  # libdab.so first (the host library links it)
        if not os.path.exists(HOST_LIB_PATH):
            raise RuntimeError(f"libdeeparc_host.so not found at {HOST_LIB_PATH}: run `make -C deeparc-sfm_amd`")
        lib = C.CDLL(HOST_LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = lib
    return _LIB


def _check(rc):
    if rc != 0:
        raise RuntimeError(load_host_library().dam_last_error().decode())


def _p(a, ct):
    return a.ctypes.data_as(C.POINTER(ct))


class DeepArcManager:
    def __init__(self):
        self.lib = load_host_library()
        h = C.c_void_p()
        _check(self.lib.dam_create(C.byref(h)))
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.dam_destroy(self.h)
            self.h = None

    def read(self, path):
        _check(self.lib.dam_read(self.h, os.fsencode(path)))
        return True

    def write(self, path):
        _check(self.lib.dam_write(self.h, os.fsencode(path)))

    def writePly(self, path):  # noqa: N802 (reference name)
        _check(self.lib.dam_write_ply(self.h, os.fsencode(path)))

    def sizes(self):
        v = [C.c_int32() for _ in range(7)]
        _check(self.lib.dam_sizes(self.h, *[C.byref(x) for x in v]))
        keys = ("blocks", "points", "intrinsics", "extrinsics", "shared", "arc", "ring")
        return dict(zip(keys, [x.value for x in v]))

    def isShareExtrinsic(self):  # noqa: N802
        return bool(self.sizes()["shared"])

    def points(self):
        n = self.sizes()["points"]
        xyz, rgb = np.zeros((n, 3)), np.zeros((n, 3), np.int32)
        _check(self.lib.dam_get_points(self.h, _p(xyz, C.c_double), _p(rgb, C.c_int32)))
        return xyz, rgb

    def cameras(self):
        s = self.sizes()
        ext, intr = np.zeros((s["extrinsics"], 6)), np.zeros((s["intrinsics"], 6))
        _check(self.lib.dam_get_cameras(self.h, _p(ext, C.c_double), _p(intr, C.c_double)))
        return ext, intr

    def blocks(self):
        n = self.sizes()["blocks"]
        a, r, pi = (np.zeros(n, np.int32) for _ in range(3))
        xy = np.zeros((n, 2))
        _check(self.lib.dam_get_blocks(self.h, _p(a, C.c_int32), _p(r, C.c_int32), _p(pi, C.c_int32),
                                       _p(xy, C.c_double)))
        return a, r, pi, xy

    def getCameraCenter(self):  # noqa: N802
        n = C.c_int32()
        _check(self.lib.dam_camera_centers(self.h, None, 0, C.byref(n)))
        out = np.zeros((n.value, 3))
        _check(self.lib.dam_camera_centers(self.h, _p(out, C.c_double), n.value, C.byref(n)))
        return out

    def filterPoint3d(self, error_boundary, hemisphere_center, hemisphere_radius):  # noqa: N802
        c = np.ascontiguousarray(hemisphere_center, np.float64)
        _check(self.lib.dam_filter(self.h, float(error_boundary), _p(c, C.c_double), float(hemisphere_radius)))


def solve(manager, max_iteration=1000, max_second=3600, freeze_camera=False,
          linear_solver_type=_abi.DAB_LINEAR_SOLVER_EXPLICIT_SCHUR):
    """sfm.cc:31 solve() on the GPU; returns the summary as a dict."""
    from .core import summary_to_dict
    its = (_abi.DabIteration * 1024)()
    s = _abi.DabSummary()
    s.iterations = C.cast(its, C.POINTER(_abi.DabIteration))
    s.iterations_capacity = 1024
    _check(manager.lib.dam_solve(manager.h, int(max_iteration), int(max_second), int(bool(freeze_camera)),
                                 int(linear_solver_type), C.byref(s)))
    return summary_to_dict(s, its)


def fit_hemisphere(centers, center=(0.0, 0.0, 0.0), radius=1.0, max_iteration=1000):
    lib = load_host_library()
    P = np.ascontiguousarray(centers, np.float64).reshape(-1, 3)
    c = np.array(center, np.float64)
    r = C.c_double(radius)
    _check(lib.dam_fit_hemisphere(_p(P, C.c_double), P.shape[0], _p(c, C.c_double), C.byref(r), max_iteration))
    return c, r.value


def run_pipeline(input_path, output_path="", ply_prefix="", max_iteration=100, max_second=3600,
                 error_boundary=5.0):
    """sfm.cc main(): fit, freeze-camera solve, filter, then solve + filter to a fixed point."""
    lib = load_host_library()
    hemi = np.zeros(4)
    counts = np.zeros(3, np.int32)
    _check(lib.dam_run_pipeline(os.fsencode(input_path), os.fsencode(output_path), os.fsencode(ply_prefix),
                                max_iteration, max_second, error_boundary, _p(hemi, C.c_double),
                                _p(counts, C.c_int32)))
    return dict(hemisphere_center=hemi[:3].copy(), hemisphere_radius=float(hemi[3]), rounds=int(counts[0]),
                blocks=int(counts[1]), points=int(counts[2]))


def run_pipeline_report(input_path, output_path="", ply_prefix="", max_iteration=100, max_second=3600,
                        error_boundary=5.0, quiet=True):
    """run_pipeline with the full report (solves, LM iterations, last cost, host timings);
    quiet suppresses the reference's per-iteration progress lines."""
    lib = load_host_library()
    r = PipelineReport()
    _check(lib.dam_run_pipeline_report(os.fsencode(input_path), os.fsencode(output_path), os.fsencode(ply_prefix),
                                       max_iteration, max_second, error_boundary, 1 if quiet else 0, C.byref(r)))
    return dict(hemisphere_center=np.array(r.hemisphere_center[:]), hemisphere_radius=r.hemisphere_radius,
                rounds=r.rounds, blocks=r.final_blocks, points=r.final_points, solves=r.solves,
                lm_iterations=r.lm_iterations, final_cost=r.final_cost, solve_seconds=r.solve_seconds,
                filter_seconds=r.filter_seconds, total_seconds=r.total_seconds,
                breakdown={k: getattr(r, k + "_seconds") for k in PIPELINE_STAGES})
