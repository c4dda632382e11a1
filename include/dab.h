/*
 * dab.h — C ABI of the MI355X bundle-adjustment solver ("dab" = DeepArc BA).
 *
 * This is the drop-in boundary that replaces the Ceres modelling/solve calls made
 * by the reference's BA driver:
 *
 *   reference (pureexe/deeparc-sfm)                     replaced by
 *   ------------------------------------------------    ------------------------------
 *   SnavelyReprojectionError::Create + AddResidualBlock  dab_problem (SoA observation
 *     src/sfm.cc:36-48, snavely_reprojection_error.hh    arrays + gather indices)
 *     :121-141, ParameterBlock::get() ParameterBlock.hh
 *     :68-94
 *   Problem::SetParameterBlockConstant  sfm.cc:50-63     dab_problem.ext_const /
 *                                                         dab_problem.freeze_camera
 *   ceres::Solver::Options  sfm.cc:66-71                 dab_options (+ dab_options_init)
 *   ceres::Solve + Summary::FullReport  sfm.cc:72-74     dab_solve + dab_summary
 *   SnavelyReprojectionError::operator()(double)         dab_eval_residuals
 *     DeepArcManager.cc:335-346 (filterPoint3d)
 *   DeepArcManager::filterPoint3d DeepArcManager.cc:     dab_filter (device residuals +
 *     332-424                                              drop masks)
 *   DynamicAutoDiffCostFunction::Evaluate (jacobians)    dab_eval_jacobians
 *     snavely_reprojection_error.hh:11-14
 *
 * Conventions: plain pointers and sizes only. The caller owns every host array. The
 * library copies the problem to the device in dab_set_problem, runs every iteration
 * device-resident, and writes the optimised `points` / `ext` back into the caller's
 * arrays when dab_solve returns (the reference's Ceres writes into the user's double*
 * blocks in place, sfm.cc:47-48). Every entry point returns 0 on success and a negative
 * DAB_E* code on error; dab_last_error() gives the message. Nothing aborts.
 * A handle is used by one host thread at a time (not re-entrant per handle).
 */
#ifndef DAB_H_
#define DAB_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DAB_ABI_VERSION 2

/* ---- status codes ---------------------------------------------------------------- */
#define DAB_OK 0
#define DAB_E_INVALID (-1)   /* bad argument / malformed problem */
#define DAB_E_DEVICE (-2)    /* HIP runtime error or no device */
#define DAB_E_NOMEM (-3)     /* device allocation failed */
#define DAB_E_STATE (-4)     /* call out of order (e.g. solve before set_problem) */
#define DAB_E_COMM (-5)      /* RCCL error */
#define DAB_E_UNSUPPORTED (-6)

/* ---- problem ----------------------------------------------------------------------
 * One residual block per observation (sfm.cc:36-48). Residual (snavely…hh:94-118):
 *   single extrinsic (ext1 < 0):   P = R(w0) X + t0
 *   composed arc∘ring (ext1 >= 0): P = R(w0) (R(w1) X + t1) + t0
 *      (ext0 = the arc extrinsic, ext1 = the ring extrinsic, snavely…hh:96-108,
 *       ParameterBlock.hh:83-87)
 *   xp = P0/P2, yp = P1/P2; d = 1 | 1+k0 r2 | 1+r2(k0+k1 r2)   (nk = 0|1|2)
 *   r = (f0 d xp + cx - x_obs,  f1' d yp + cy - y_obs),  f1' = nf==2 ? f1 : f0
 * Extrinsic layout: ext[e] = (w0,w1,w2, t0,t1,t2) — angle-axis rotation then
 * translation (the two 3-blocks of Extrinsic.hh:32).
 * Intrinsic layout: intr[i] = (cx, cy, f0, f1, k0, k1) with intr_nf[i] in {1,2},
 * intr_nk[i] in {0,1,2} (Intrinsic.hh:32; unused slots ignored).
 * Intrinsics are never optimised (sfm.cc:54-63).
 * Constancy: points are free; an extrinsic is free unless ext_const[e] != 0 or
 * freeze_camera != 0 (sfm.cc:50-57). Parameter blocks referenced by no observation
 * are not part of the problem (Ceres only knows blocks added via AddResidualBlock)
 * and are left untouched.
 */
typedef struct dab_problem {
  int32_t num_obs;
  int32_t num_points;
  int32_t num_ext;
  int32_t num_intr;
  const double* obs_xy;      /* [num_obs][2] observed pixel (Point2d, Point2d.hh:12) */
  const int32_t* obs_point;  /* [num_obs] point index */
  const int32_t* obs_ext0;   /* [num_obs] extrinsic (arc when composed) */
  const int32_t* obs_ext1;   /* [num_obs] ring extrinsic when composed, else -1 */
  const int32_t* obs_intr;   /* [num_obs] intrinsic index */
  double* points;            /* [num_points][3] in/out */
  double* ext;               /* [num_ext][6] in/out */
  const double* intr;        /* [num_intr][6] */
  const int32_t* intr_nf;    /* [num_intr] */
  const int32_t* intr_nk;    /* [num_intr] */
  const uint8_t* ext_const;  /* [num_ext] or NULL */
  int32_t freeze_camera;     /* solve(..., freeze_camera=true), sfm.cc:54-57 */
  int32_t reserved;
} dab_problem;

/* ---- options (mirrors the ceres::Solver::Options fields the reference uses plus the
 * Ceres trust-region defaults it relies on implicitly) ------------- */
#define DAB_LINEAR_SOLVER_EXPLICIT_SCHUR 0  /* exact: DENSE_SCHUR equivalent (sfm.cc:67) */
#define DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG 1 /* inexact: ITERATIVE_SCHUR + SCHUR_JACOBI */
/* the exact step where it scales over the ranks, PCG where it does not: EXPLICIT_SCHUR on
 * one rank and, on several, for small camera systems (<= 160 free cameras: the rig; S is a
 * few MB to all-reduce and its factorisation takes microseconds); IMPLICIT_SCHUR_PCG for
 * large camera systems on several ranks (BASELINE config 4: the 288-MB S all-reduce and the
 * serial 5.5-ms factorisation on every rank would cap the speed-up near 1.2x). The summary's
 * linear_solver_type_used says which ran. */
#define DAB_LINEAR_SOLVER_AUTO 2

typedef struct dab_options {
  int32_t max_num_iterations;            /* sfm.cc:69 (call sites pass 100) */
  int32_t linear_solver_type;            /* DAB_LINEAR_SOLVER_* */
  double max_solver_time_in_seconds;     /* sfm.cc:71 */
  double function_tolerance;             /* 1e-6 */
  double gradient_tolerance;             /* 1e-10 */
  double parameter_tolerance;            /* 1e-8 */
  double min_relative_decrease;          /* 1e-3 */
  double initial_trust_region_radius;    /* 1e4 */
  double max_trust_region_radius;        /* 1e16 */
  double min_trust_region_radius;        /* 1e-32 */
  double min_lm_diagonal;                /* 1e-6 */
  double max_lm_diagonal;                /* 1e32 */
  int32_t max_num_consecutive_invalid_steps; /* 5 */
  int32_t jacobi_scaling;                /* 1 */
  int32_t minimizer_progress_to_stdout;  /* sfm.cc:68 */
  int32_t num_threads;                   /* CPU paths only (sfm.cc:70) */
  /* PCG (IMPLICIT_SCHUR_PCG only) — Ceres ITERATIVE_SCHUR defaults */
  int32_t max_linear_solver_iterations;  /* 500 */
  int32_t min_linear_solver_iterations;  /* 0 */
  double eta;                            /* 1e-1 (Nash–Sofer q-tolerance) */
  int32_t pcg_fp32;                      /* 1: fp32 matvec/preconditioner, fp64 accumulate */
  int32_t reserved;
} dab_options;

/* ---- summary (ceres::Solver::Summary subset, sfm.cc:72-74) ------------------------ */
#define DAB_CONVERGENCE 0
#define DAB_NO_CONVERGENCE 1
#define DAB_FAILURE 2

typedef struct dab_iteration {
  int32_t iteration;
  int32_t step_is_successful;
  int32_t step_is_valid;
  int32_t linear_solver_iterations;
  double cost;
  double cost_change;
  double gradient_max_norm;
  double step_norm;
  double relative_decrease;
  double trust_region_radius;
  double iteration_time_in_seconds;
} dab_iteration;

typedef struct dab_summary {
  double initial_cost;
  double final_cost;
  int32_t num_iterations;          /* index of the last iteration record */
  int32_t num_successful_steps;    /* iteration 0 counts, as in Ceres */
  int32_t num_unsuccessful_steps;
  int32_t termination_type;        /* DAB_CONVERGENCE / NO_CONVERGENCE / FAILURE */
  int32_t num_residuals;
  int32_t num_parameters;          /* free scalar parameters */
  int32_t num_free_points;
  int32_t num_free_ext;
  double total_time_in_seconds;
  double jacobian_evaluation_time_in_seconds;
  double residual_evaluation_time_in_seconds;
  double linear_solver_time_in_seconds;
  char message[256];
  dab_iteration* iterations;       /* optional caller buffer (may be NULL) */
  int32_t iterations_capacity;     /* entries available in `iterations` */
  int32_t iterations_written;      /* entries filled */
  int32_t linear_solver_type_used; /* the DAB_LINEAR_SOLVER_* that ran (the requested one, or
                                      what DAB_LINEAR_SOLVER_AUTO chose) */
  int32_t schur_assembly;          /* EXPLICIT_SCHUR: DAB_SCHUR_* (how S was assembled);
                                      IMPLICIT_SCHUR_PCG: DAB_PCG_* (the Schur products) */
} dab_summary;
/* schur_assembly values for DAB_LINEAR_SOLVER_EXPLICIT_SCHUR */
#define DAB_SCHUR_PAIRS 0   /* per camera-pair block sums over entry-pair tables (large NC) */
#define DAB_SCHUR_TILES 1   /* register-owned block tiles over per-step Y records (NC <= 160) */
/* schur_assembly values for DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG */
#define DAB_PCG_STORED_Y 0          /* products over stored Y records (fp32 records with pcg_fp32) */
#define DAB_PCG_MATRIX_FREE 1       /* rows re-evaluated per product, all fp64 (NC <= 160) */
#define DAB_PCG_MATRIX_FREE_FP32 2  /* as 1 with pcg_fp32: fp32 per-observation arithmetic, fp64
                                       sums, fp64 CG recurrences and true residuals */

typedef struct dab_handle dab_handle;

/* ---- lifecycle ---------------------------------------------------------------------- */
int dab_abi_version(void);
const char* dab_last_error(void);
void dab_options_init(dab_options* opt);

/* device: HIP ordinal. Single-process handle (world_size 1).
   Side effect, process-wide: every dab_create* sets hipSetDeviceFlags(hipDeviceScheduleSpin)
   (the LM loop's host round trips are latency-critical), so every host wait of the
   embedding process spins instead of blocking. DAB_SCHEDULE_BLOCKING=1 in the environment
   keeps the runtime's default; a refused flag is reported once on stderr. */
int dab_create(int device, dab_handle** out);
/* Multi-GPU (one process per GPU, RCCL over xGMI). `unique_id` is the 128-byte
 * ncclUniqueId produced on rank 0 by dab_comm_unique_id and broadcast by the caller.
 * world_size 1 with a non-null unique_id builds a one-rank RCCL communicator and runs
 * the solve's collectives through it — the evaluation pass's (the split schedule with its
 * camera all-reduce on the communication stream included), the LM step's and every PCG
 * iteration's: the same results as dab_create, with the multi-GPU transport executed on one
 * GPU. The set-up's free-camera and pair-set unions, the LINEAR_SOLVER_AUTO choice and the
 * rig's matrix-free PCG product (whose work-group partials a single rank sums inside the CG
 * update, no all-reduce) follow world_size, so they take the one-rank paths. */
int dab_comm_unique_id(uint8_t out_id[128]);
int dab_create_dist(int device, int rank, int world_size, const uint8_t unique_id[128],
                    dab_handle** out);
/* Host-staged collective, for rehearsing the multi-rank path where RCCL cannot run
 * (several ranks sharing one GPU; CI). Every all-reduce copies the device buffer to
 * host memory and calls cb(buf, count, op, user), which must reduce it in place across
 * the ranks (op 0 = sum, 1 = max; e.g. over gloo) and return 0. Not the product path:
 * one process per GPU uses dab_create_dist (RCCL over xGMI). */
typedef int (*dab_host_allreduce_fn)(double* buf, int64_t count, int op, void* user);
int dab_create_dist_host(int device, int rank, int world_size, dab_host_allreduce_fn cb, void* user,
                         dab_handle** out);
/* Frees the handle's device buffers. Its streams and small pinned host blocks go to a
 * process-wide cache that the next dab_create on the same device takes from (creating and
 * destroying a stream cost ~2 ms each); a cached stream that reports an error is destroyed
 * instead of reused. */
int dab_destroy(dab_handle* h);
/* Destroys the cached streams and frees the cached pinned blocks (an embedding process that
 * resets the device, or wants the memory back). Safe with handles alive: it touches only
 * the idle objects in the cache, never a live handle's own streams or pinned blocks (each
 * stream is destroyed with its own device current, the caller's device restored). To get
 * every stream back, destroy the handles first. */
int dab_release_caches(void);

/* ---- problem upload / solve ------------------------------------------------------------
 * dab_set_problem copies the problem to the device and builds the point-major and
 * camera-major orderings once. In a multi-GPU handle each rank passes its own shard
 * (observations of a disjoint point set; extrinsics and intrinsics replicated with
 * identical values on every rank). */
int dab_set_problem(dab_handle* h, const dab_problem* p);
/* Re-upload only the parameter values (points, ext) of the current problem. */
int dab_update_parameters(dab_handle* h, const double* points, const double* ext);
int dab_solve(dab_handle* h, const dab_options* opt, dab_summary* summary);
/* Copy the device-resident parameters into host arrays (either may be NULL). */
int dab_get_parameters(dab_handle* h, double* points, double* ext);

/* ---- evaluation (parity / filterPoint3d) ---------------------------------------------
 * residuals: [num_obs][2] in the caller's observation order.
 * jacobians: [num_obs][2][15] row-major, columns = [X(3) | w0(3) t0(3) | w1(3) t1(3)]
 *            (d r / d param, unscaled; w1/t1 columns are zero for single-extrinsic obs).
 * cost: 0.5 * sum r^2. Any pointer may be NULL. */
int dab_eval_residuals(dab_handle* h, double* residuals, double* cost);
int dab_eval_jacobians(dab_handle* h, double* residuals, double* jacobians);

/* DeepArcManager::filterPoint3d (DeepArcManager.cc:332-424) on the device, at the
 * parameters currently on the handle (after dab_solve: the optimised ones):
 *   1. an observation is dropped when mse = (r0^2 + r1^2) / 2 < error_boundary
 *      (quirk Q4: the *small*-error ones, exactly as the reference);
 *   2. a point with no remaining observation is dropped (Point3d::empty);
 *   3. a remaining point is dropped when |X - center|^2 > radius / 2 (radius is the
 *      fitted *squared* radius, hemisphere_radius.hh:26), and so are its observations.
 * obs_keep[num_obs] and point_keep[num_points] (caller order; 1 = kept) may be NULL;
 * unreferenced points are reported as dropped. Counts of kept items in *n_obs_kept /
 * *n_points_kept (nullable). The handle's problem is not modified. */
int dab_filter(dab_handle* h, double error_boundary, const double center[3], double radius,
               uint8_t* obs_keep, uint8_t* point_keep, int32_t* n_obs_kept, int32_t* n_points_kept);

/* Dense SPD solve A x = b on the handle's device with the library's blocked Cholesky (the
 * reduced-camera-system factorisation of DAB_LINEAR_SOLVER_EXPLICIT_SCHUR; Eigen LLT in
 * Ceres' DENSE_SCHUR). A: n x n row-major, only the lower triangle is read. factor_ms
 * (nullable): device time of factorisation + solves. Returns DAB_OK, 1 when A is not
 * numerically positive definite, or a negative error. */
int dab_dense_spd_solve(dab_handle* h, int n, const double* A, const double* b, double* x,
                        double* factor_ms);

/* ---- benchmark hooks -------------------------------------------------------------------
 * `count` evaluation passes on device-resident data, enqueued back to back: residual +
 * Jacobian with the JtJ / Jtr block assembly (per-point V,g and per-camera U,g, all-reduced
 * across ranks). Asynchronous on the handle's stream; dab_sync waits for them. One call per
 * batch keeps the host's launch cost off the device's critical path. */
int dab_bench_eval_pass(dab_handle* h, int with_assembly, int count);
int dab_sync(dab_handle* h);
/* Kernel timing: average device time (ms) of the point-side residual+Jacobian kernel and
 * of the rest of the pass, over the passes since the last call, measured with HIP events on
 * the handle's stream (every 8th pass of a dab_bench_eval_pass batch and its first one;
 * environment DAB_BENCH_SAMPLE sets the stride). */
int dab_bench_kernel_ms(dab_handle* h, double* jac_ms, double* assembly_ms);
/* Algorithmic HBM bytes of one residual+Jacobian launch on the resident problem. */
int dab_jacobian_bytes(dab_handle* h, double* bytes);
/* The rig's pair-major camera kernel (k_eval_pair; composed observations with both
 * cameras free): its average device time (ms) over the sampled passes of the batches read
 * by the last dab_bench_kernel_ms call, and its algorithmic bytes per launch (0 when the
 * resident problem has no pair-major pass). */
int dab_bench_pair_ms(dab_handle* h, double* ms, double* bytes);
/* Which evaluation schedule the resident problem uses: *fused = 1 when the pass is the
 * single fused launch (k_eval_fused: camera and point side together), 2 when it is the
 * same kernel as a camera-side then a point-side launch (several ranks: the camera blocks'
 * all-reduce overlaps the point side), 0 for the two-kernel pass (k_eval_cams +
 * k_eval_points). */
int dab_eval_schedule(dab_handle* h, int32_t* fused);
/* After an IMPLICIT_SCHUR_PCG solve: *matrix_free = 1 when the Schur products re-evaluate
 * the observation rows in every pass (small camera sets, fp64, no Y records), 2 for the
 * same with pcg_fp32 (fp32 per-observation arithmetic, fp64 sums and true residuals), 0 for
 * the stored-Y products. */
int dab_pcg_schedule(dab_handle* h, int32_t* matrix_free);
/* How the handle's sums over ranks run: *p2p = 1 when the one-shot peer-to-peer all-reduce
 * over xGMI (IPC-mapped peer regions, fixed rank order) carries the camera-sized sums (every
 * pair of devices peer-accessible; environment DAB_P2P=0 disables it, DAB_P2P=1 also enables
 * it on host-staged handles), 0 when every collective is RCCL or host-staged. */
int dab_comm_schedule(dab_handle* h, int32_t* p2p);

/* ---- host utilities (no device needed) ----------------------------------------------- */
/* Deterministic synthetic problems. kind 0: BAL-shaped (non-shared, one
 * intrinsic per camera); kind 1: DeepArc rig (arcs x rings, shared intrinsics).
 * Query sizes with arrays NULL, then call again with caller-allocated arrays. */
typedef struct dab_synth_config {
  int32_t kind;          /* 0 BAL-shaped, 1 rig */
  int32_t num_cameras;   /* kind 0 */
  int32_t num_arcs;      /* kind 1 */
  int32_t num_rings;     /* kind 1 */
  int32_t num_points;
  int32_t obs_per_point;
  uint64_t seed;         /* cameras, intrinsics and their initial values */
  uint64_t point_seed;   /* points/observations stream; 0 = continue the `seed` stream.
                            Shards of one global problem share `seed` and differ here. */
  double pixel_noise;    /* 1.0 */
  double point_noise;    /* 0.01 */
  double rot_noise;      /* 1e-3 */
  double trans_noise;    /* 1e-3 */
} dab_synth_config;

int dab_synth_sizes(const dab_synth_config* cfg, int32_t* num_obs, int32_t* num_points,
                    int32_t* num_ext, int32_t* num_intr);
/* Fills the arrays of `p` (sizes must match dab_synth_sizes). ext_const gets the
 * gauge rule of sfm.cc:50-53. */
int dab_synth_fill(const dab_synth_config* cfg, dab_problem* p, uint8_t* ext_const);

#ifdef __cplusplus
}
#endif
#endif /* DAB_H_ */
