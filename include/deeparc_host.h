/*
 * deeparc_host.h — C ABI of the host adapter (deeparc-sfm_amd/host, libdeeparc_host.so).
 *
 * The C++ API in deeparc-sfm_amd/host mirrors the reference's host classes
 * (DeepArcManager, ParameterBlock, Point3d, Intrinsic, Extrinsic, Camera) and the driver
 * functions of src/sfm.cc (solve, the hemisphere fit, the solve -> filterPoint3d loop)
 * over libdab. This flat C layer exists for bindings and tests (ctypes); each function
 * names the reference call it wraps:
 *   dam_read / dam_write / dam_write_ply   DeepArcManager::read / write / writePly
 *                                          (DeepArcManager.cc:26-196, 426-499, 263-328)
 *   dam_solve                              solve(DeepArcManager&, ...), sfm.cc:31-75
 *   dam_filter                             DeepArcManager::filterPoint3d, DeepArcManager.cc:332-424
 *   dam_camera_centers                     DeepArcManager::getCameraCenter, DeepArcManager.cc:501-518
 *   dam_fit_hemisphere                     the HemisphereRadius fit, sfm.cc:83-101
 *   dam_run_pipeline                       main(), sfm.cc:79-129
 * Return 0 on success, negative on error (message in dam_last_error; the C++ API throws
 * const char* like the reference).
 */
#ifndef DEEPARC_HOST_H_
#define DEEPARC_HOST_H_

#include <stdint.h>

#include "dab.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dam_manager dam_manager;

const char* dam_last_error(void);
int dam_create(dam_manager** out);
int dam_destroy(dam_manager* m);
int dam_read(dam_manager* m, const char* path);
int dam_write(dam_manager* m, const char* path);
int dam_write_ply(dam_manager* m, const char* path);
/* sizes of the current scene; shared = rig mode (n_ring != 0) */
int dam_sizes(dam_manager* m, int32_t* n_blocks, int32_t* n_points, int32_t* n_intr, int32_t* n_ext,
              int32_t* shared, int32_t* n_arc, int32_t* n_ring);
/* xyz [n_points][3], rgb [n_points][3] (either may be NULL) */
int dam_get_points(dam_manager* m, double* xyz, int32_t* rgb);
/* ext [n_ext][6] = (w, t); intr [n_intr][6] = (cx, cy, f0, f1, k0, k1) (either may be NULL) */
int dam_get_cameras(dam_manager* m, double* ext, double* intr);
/* per block: pos_arc, pos_ring, index of its point in the current point list, (x, y) */
int dam_get_blocks(dam_manager* m, int32_t* pos_arc, int32_t* pos_ring, int32_t* point_index, double* xy);
/* solve(m, max_iteration, max_second, freeze_camera) with the given linear solver;
 * summary may be NULL */
int dam_solve(dam_manager* m, int32_t max_iteration, int32_t max_second, int32_t freeze_camera,
              int32_t linear_solver_type, dab_summary* summary);
int dam_filter(dam_manager* m, double error_boundary, const double center[3], double radius);
/* out [capacity][3]; *count = number of centres (may exceed capacity) */
int dam_camera_centers(dam_manager* m, double* out, int32_t capacity, int32_t* count);
/* centres [n][3]; center/radius are the starting point on input, the fit on output */
int dam_fit_hemisphere(const double* centers, int32_t n, double center[3], double* radius,
                       int32_t max_iteration);
/* hemi_out = (cx, cy, cz, R); counts_out = (rounds, blocks, points); output / ply_prefix
 * may be empty strings */
int dam_run_pipeline(const char* input, const char* output, const char* ply_prefix, int32_t max_iteration,
                     int32_t max_second, double error_boundary, double hemi_out[4], int32_t counts_out[3]);
/* the same loop with a full report; quiet != 0 suppresses the per-iteration progress and
 * the per-solve summary lines the reference prints */
typedef struct dam_pipeline_report {
  double hemisphere_center[3], hemisphere_radius;
  int32_t rounds, final_blocks, final_points, solves;
  int32_t lm_iterations, reserved;  /* LM iterations summed over the solves */
  double final_cost;                /* the last solve's final cost */
  double solve_seconds, filter_seconds, total_seconds;
  /* breakdown, seconds summed over the loop: .deeparc read, hemisphere fit, PLY/output
   * writes; per libdab handle stage: marshal (manager -> SoA arrays), setup
   * (dab_set_problem), update (values-only refresh), prep (a solve's table build and graph
   * capture), lm (the LM iterations), writeback, filter device pass, filter host compaction */
  double read_seconds, fit_seconds, write_seconds, marshal_seconds, setup_seconds, update_seconds, prep_seconds,
      lm_seconds, writeback_seconds, filter_device_seconds, filter_host_seconds;
} dam_pipeline_report;
int dam_run_pipeline_report(const char* input, const char* output, const char* ply_prefix, int32_t max_iteration,
                            int32_t max_second, double error_boundary, int32_t quiet, dam_pipeline_report* out);

#ifdef __cplusplus
}
#endif
#endif
