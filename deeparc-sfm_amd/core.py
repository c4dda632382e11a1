"""Python host mirror of the reference BA interface over the C ABI (libdab.so).

Mirrors (names, argument meaning, error behaviour) of the reference:
  solve(manager_or_problem, max_iteration=1000, max_second=3600, freeze_camera=False)
      src/sfm.cc:31-75 — builds the problem from the observation -> parameter mapping
      (ParameterBlock::get(), ParameterBlock.hh:68-94), applies the gauge / constancy
      rules (sfm.cc:50-63) and solves with the DENSE_SCHUR-equivalent solver
      (sfm.cc:66-73). Parameters are updated in place, as Ceres does.
  Problem.residuals()   — SnavelyReprojectionError::operator()(double) per observation
      (DeepArcManager.cc:335-346)
The heavy lifting is the gfx950 HIP library; this module only marshals numpy arrays.
"""
import ctypes as C

import numpy as np

from . import _abi
from ._abi import (DabOptions, DabProblem, DabSummary, DabIteration, DabSynthConfig, check,
                   load_library)


def _ptr(a, ct):
    return a.ctypes.data_as(C.POINTER(ct)) if a is not None else None


class Problem:
    """SoA bundle-adjustment problem (the dab_problem of include/dab.h) backed by numpy."""

    def __init__(self, obs_xy, obs_point, obs_ext0, obs_ext1, obs_intr, points, ext, intr,
                 intr_nf, intr_nk, ext_const=None, freeze_camera=False):
        self.obs_xy = np.ascontiguousarray(obs_xy, dtype=np.float64).reshape(-1, 2)
        self.obs_point = np.ascontiguousarray(obs_point, dtype=np.int32)
        self.obs_ext0 = np.ascontiguousarray(obs_ext0, dtype=np.int32)
        self.obs_ext1 = np.ascontiguousarray(obs_ext1, dtype=np.int32)
        self.obs_intr = np.ascontiguousarray(obs_intr, dtype=np.int32)
        self.points = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
        self.ext = np.ascontiguousarray(ext, dtype=np.float64).reshape(-1, 6)
        self.intr = np.ascontiguousarray(intr, dtype=np.float64).reshape(-1, 6)
        self.intr_nf = np.ascontiguousarray(intr_nf, dtype=np.int32)
        self.intr_nk = np.ascontiguousarray(intr_nk, dtype=np.int32)
        self.ext_const = (np.ascontiguousarray(ext_const, dtype=np.uint8)
                          if ext_const is not None else None)
        self.freeze_camera = bool(freeze_camera)

    @property
    def num_obs(self):
        return int(self.obs_point.shape[0])

    def copy(self):
        return Problem(self.obs_xy.copy(), self.obs_point.copy(), self.obs_ext0.copy(),
                       self.obs_ext1.copy(), self.obs_intr.copy(), self.points.copy(),
                       self.ext.copy(), self.intr.copy(), self.intr_nf.copy(),
                       self.intr_nk.copy(),
                       None if self.ext_const is None else self.ext_const.copy(),
                       self.freeze_camera)

    def subset(self, obs_mask):
        """Observations selected by obs_mask; parameter arrays are shared (not copied)."""
        m = np.asarray(obs_mask)
        return Problem(self.obs_xy[m], self.obs_point[m], self.obs_ext0[m], self.obs_ext1[m],
                       self.obs_intr[m], self.points, self.ext, self.intr, self.intr_nf,
                       self.intr_nk, self.ext_const, self.freeze_camera)

    def point_owner(self, world):
        """Owner rank of every point for a world-size sharding (partition by
        point, so V, V^-1 and the back-substitution stay GPU-local): contiguous point-id
        ranges whose observation counts are balanced. Cameras are replicated."""
        npts = int(self.points.shape[0])
        cnt = np.bincount(self.obs_point, minlength=npts).astype(np.int64)
        total = int(cnt.sum())
        start = np.cumsum(cnt) - cnt
        return np.minimum(start * world // max(total, 1), world - 1).astype(np.int32)

    def shard(self, rank, world):
        """The observations of the points owned by `rank` (parameter arrays shared, the
        gauge / ext_const of the global problem kept)."""
        if world <= 1:
            return self
        owner = self.point_owner(world)
        return self.subset(owner[self.obs_point] == rank)

    def as_c(self):
        """dab_problem view of the arrays (valid while self is alive)."""
        p = DabProblem()
        p.num_obs = self.num_obs
        p.num_points = int(self.points.shape[0])
        p.num_ext = int(self.ext.shape[0])
        p.num_intr = int(self.intr.shape[0])
        p.obs_xy = _ptr(self.obs_xy, C.c_double)
        p.obs_point = _ptr(self.obs_point, C.c_int32)
        p.obs_ext0 = _ptr(self.obs_ext0, C.c_int32)
        p.obs_ext1 = _ptr(self.obs_ext1, C.c_int32)
        p.obs_intr = _ptr(self.obs_intr, C.c_int32)
        p.points = _ptr(self.points, C.c_double)
        p.ext = _ptr(self.ext, C.c_double)
        p.intr = _ptr(self.intr, C.c_double)
        p.intr_nf = _ptr(self.intr_nf, C.c_int32)
        p.intr_nk = _ptr(self.intr_nk, C.c_int32)
        p.ext_const = _ptr(self.ext_const, C.c_uint8) if self.ext_const is not None else None
        p.freeze_camera = int(self.freeze_camera)
        return p


def synth_config(kind=0, num_cameras=0, num_arcs=0, num_rings=0, num_points=0,
                 obs_per_point=10, seed=1, point_seed=0, pixel_noise=1.0, point_noise=0.01,
                 rot_noise=1e-3, trans_noise=1e-3):
    c = DabSynthConfig()
    c.kind, c.num_cameras, c.num_arcs, c.num_rings = kind, num_cameras, num_arcs, num_rings
    c.num_points, c.obs_per_point, c.seed, c.point_seed = num_points, obs_per_point, seed, point_seed
    c.pixel_noise, c.point_noise, c.rot_noise, c.trans_noise = (pixel_noise, point_noise,
                                                                rot_noise, trans_noise)
    return c


def synth(**kw):
    """Deterministic synthetic problem generated by libdab's host code."""
    lib = load_library()
    cfg = synth_config(**kw)
    no, npt, ne, ni = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int32()
    check(lib.dab_synth_sizes(C.byref(cfg), C.byref(no), C.byref(npt), C.byref(ne),
                              C.byref(ni)), lib)
    no, npt, ne, ni = no.value, npt.value, ne.value, ni.value
    pr = Problem(np.zeros((no, 2)), np.zeros(no, np.int32), np.zeros(no, np.int32),
                 np.zeros(no, np.int32), np.zeros(no, np.int32), np.zeros((npt, 3)),
                 np.zeros((ne, 6)), np.zeros((ni, 6)), np.zeros(ni, np.int32),
                 np.zeros(ni, np.int32), np.zeros(ne, np.uint8))
    cp = pr.as_c()
    check(lib.dab_synth_fill(C.byref(cfg), C.byref(cp), _ptr(pr.ext_const, C.c_uint8)), lib)
    return pr


# SURVEY §8d named configurations
CONFIGS = {
    "c1_rig_8x36": dict(kind=1, num_arcs=8, num_rings=36, num_points=20000, obs_per_point=8, seed=4),
    "c2_100cam": dict(kind=0, num_cameras=100, num_points=10000, obs_per_point=10, seed=1),
    "c3_1kcam": dict(kind=0, num_cameras=1000, num_points=100000, obs_per_point=10, seed=2),
    "c5_rig_16x64": dict(kind=1, num_arcs=16, num_rings=64, num_points=1000000,
                         obs_per_point=10, seed=3),
}


def options(**kw):
    lib = load_library()
    o = DabOptions()
    lib.dab_options_init(C.byref(o))
    for k, v in kw.items():
        if not hasattr(o, k):
            raise AttributeError(f"unknown option {k}")
        setattr(o, k, v)
    return o


def summary_to_dict(s, its):
    return dict(
        initial_cost=s.initial_cost, final_cost=s.final_cost, num_iterations=s.num_iterations,
        num_successful_steps=s.num_successful_steps,
        num_unsuccessful_steps=s.num_unsuccessful_steps,
        termination=_abi.TERMINATION.get(s.termination_type, str(s.termination_type)),
        message=s.message.decode(errors="replace"), num_residuals=s.num_residuals,
        num_parameters=s.num_parameters, num_free_points=s.num_free_points,
        num_free_ext=s.num_free_ext, total_time=s.total_time_in_seconds,
        jacobian_time=s.jacobian_evaluation_time_in_seconds,
        residual_time=s.residual_evaluation_time_in_seconds,
        linear_solver_time=s.linear_solver_time_in_seconds,
        linear_solver_type_used=s.linear_solver_type_used, schur_assembly=s.schur_assembly,
        iterations=[dict(iteration=it.iteration, success=bool(it.step_is_successful),
                         valid=bool(it.step_is_valid), cost=it.cost, cost_change=it.cost_change,
                         gradient_max_norm=it.gradient_max_norm, step_norm=it.step_norm,
                         relative_decrease=it.relative_decrease,
                         trust_region_radius=it.trust_region_radius,
                         linear_solver_iterations=it.linear_solver_iterations,
                         time=it.iteration_time_in_seconds)
                    for it in its[: s.iterations_written]])


class Solver:
    """One libdab handle (one GPU). For multi-GPU pass rank/world/unique_id (RCCL).

    host_allreduce (rehearsal only): a callable(np.ndarray, op) that all-reduces the array
    in place across ranks (op "sum" | "max"), e.g. over gloo; the library then stages its
    collectives through host memory instead of RCCL, so several ranks may share one GPU."""

    def __init__(self, device=0, rank=0, world_size=1, unique_id=None, host_allreduce=None):
        self.lib = load_library()
        h = C.c_void_p()
        self._cb = None
        if world_size > 1 and host_allreduce is not None:
            def _cb(buf, count, op, user):
                try:
                    arr = np.ctypeslib.as_array(buf, shape=(int(count),))
                    host_allreduce(arr, "max" if op == 1 else "sum")
                    return 0
                except Exception:  # reported to the library as a collective failure
                    return 1
            self._cb = _abi.HostAllreduceFn(_cb)
            check(self.lib.dab_create_dist_host(device, rank, world_size, self._cb, None, C.byref(h)),
                  self.lib)
        elif world_size > 1 or unique_id is not None:
            # world_size 1 with a unique id: a one-rank RCCL communicator, every collective
            # executed (the multi-GPU transport rehearsed on one GPU)
            buf = (C.c_uint8 * 128).from_buffer_copy(bytes(unique_id))
            check(self.lib.dab_create_dist(device, rank, world_size, buf, C.byref(h)), self.lib)
        else:
            check(self.lib.dab_create(device, C.byref(h)), self.lib)
        self.h = h
        self.problem = None
        self._cp = None

    @staticmethod
    def unique_id():
        lib = load_library()
        buf = (C.c_uint8 * 128)()
        check(lib.dab_comm_unique_id(buf), lib)
        return bytes(buf)

    def close(self):
        if self.h:
            self.lib.dab_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_problem(self, problem):
        self.problem = problem
        self._cp = problem.as_c()
        check(self.lib.dab_set_problem(self.h, C.byref(self._cp)), self.lib)

    def update_parameters(self, points=None, ext=None):
        check(self.lib.dab_update_parameters(
            self.h, _ptr(np.ascontiguousarray(points, np.float64), C.c_double) if points is not None else None,
            _ptr(np.ascontiguousarray(ext, np.float64), C.c_double) if ext is not None else None), self.lib)

    def solve(self, opts=None, max_records=1024):
        o = opts if opts is not None else options()
        its = (DabIteration * max_records)()
        s = DabSummary()
        s.iterations = C.cast(its, C.POINTER(DabIteration))
        s.iterations_capacity = max_records
        check(self.lib.dab_solve(self.h, C.byref(o), C.byref(s)), self.lib)
        return summary_to_dict(s, its)

    def residuals(self):
        r = np.zeros((self.problem.num_obs, 2))
        cost = C.c_double()
        check(self.lib.dab_eval_residuals(self.h, _ptr(r, C.c_double), C.byref(cost)), self.lib)
        return r, cost.value

    def jacobians(self):
        n = self.problem.num_obs
        r = np.zeros((n, 2))
        J = np.zeros((n, 2, 15))
        check(self.lib.dab_eval_jacobians(self.h, _ptr(r, C.c_double), _ptr(J, C.c_double)),
              self.lib)
        return r, J

    def filter(self, error_boundary, center, radius):
        """filterPoint3d's masks on the resident problem (dab_filter): (observation keep,
        point keep) in the caller's order, uint8."""
        ok = np.zeros(self.problem.num_obs, np.uint8)
        pk = np.zeros(self.problem.points.shape[0], np.uint8)
        c = np.ascontiguousarray(center, np.float64)
        check(self.lib.dab_filter(self.h, float(error_boundary), _ptr(c, C.c_double), float(radius),
                                  _ptr(ok, C.c_uint8), _ptr(pk, C.c_uint8), None, None), self.lib)
        return ok, pk

    def get_parameters(self, points, ext):
        check(self.lib.dab_get_parameters(self.h, _ptr(points, C.c_double), _ptr(ext, C.c_double)),
              self.lib)

    def dense_spd_solve(self, A, b):
        """Solve A x = b with the library's device Cholesky. Returns (x, ms, ok)."""
        A = np.ascontiguousarray(A, np.float64)
        b = np.ascontiguousarray(b, np.float64)
        x = np.zeros(b.shape[0])
        ms = C.c_double()
        rc = self.lib.dab_dense_spd_solve(self.h, int(b.shape[0]), _ptr(A, C.c_double),
                                          _ptr(b, C.c_double), _ptr(x, C.c_double), C.byref(ms))
        if rc < 0:
            check(rc, self.lib)
        return x, ms.value, rc == 0

    # --- benchmark hooks ---
    def bench_eval_pass(self, with_assembly=True, count=1):
        """Enqueue `count` evaluation passes (asynchronous; sync() waits)."""
        check(self.lib.dab_bench_eval_pass(self.h, int(with_assembly), int(count)), self.lib)

    def sync(self):
        check(self.lib.dab_sync(self.h), self.lib)

    def bench_kernel_ms(self):
        a, b = C.c_double(), C.c_double()
        check(self.lib.dab_bench_kernel_ms(self.h, C.byref(a), C.byref(b)), self.lib)
        return a.value, b.value

    def jacobian_bytes(self):
        b = C.c_double()
        check(self.lib.dab_jacobian_bytes(self.h, C.byref(b)), self.lib)
        return b.value

    def bench_pair_ms(self):
        """(ms per launch, algorithmic bytes per launch) of the rig's pair-major camera kernel
        over the batches read by the last bench_kernel_ms() call"""
        a, b = C.c_double(), C.c_double()
        check(self.lib.dab_bench_pair_ms(self.h, C.byref(a), C.byref(b)), self.lib)
        return a.value, b.value

    def comm_p2p(self):
        """1 when the one-shot xGMI peer-to-peer all-reduce carries the sums over ranks"""
        f = C.c_int32()
        check(self.lib.dab_comm_schedule(self.h, C.byref(f)), self.lib)
        return int(f.value)

    def pcg_matrix_free(self):
        """0: stored-Y products; 1: matrix-free fp64; 2: matrix-free mixed precision (pcg_fp32)"""
        f = C.c_int32()
        check(self.lib.dab_pcg_schedule(self.h, C.byref(f)), self.lib)
        return int(f.value)

    def eval_fused(self):
        f = C.c_int32()
        check(self.lib.dab_eval_schedule(self.h, C.byref(f)), self.lib)
        return f.value  # 0 two kernels, 1 one fused launch, 2 fused kernel split per side


def solve(problem, max_iteration=1000, max_second=3600, freeze_camera=False, device=0,
          verbose=False, **opt_kw):
    """Drop-in for the reference's solve() (src/sfm.cc:31): DENSE_SCHUR-equivalent LM,
    max_num_iterations / max_solver_time_in_seconds as given, parameters updated in place."""
    problem.freeze_camera = bool(freeze_camera)
    o = options(max_num_iterations=max_iteration, max_solver_time_in_seconds=float(max_second),
                minimizer_progress_to_stdout=int(verbose), **opt_kw)
    s = Solver(device)
    try:
        s.set_problem(problem)
        return s.solve(o)
    finally:
        s.close()
