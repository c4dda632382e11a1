// sfm.hh — the reference's driver functions over libdab (src/sfm.cc):
//   solve()         replaces the Ceres problem of sfm.cc:31-75 (same arguments,
//                   same constancy / gauge rules, parameters updated in place);
//   fitHemisphere() replaces the HemisphereRadius fit of sfm.cc:83-101
//                   (hemisphere_radius.hh: r_i = |c - p_i|^2 - R, a squared radius);
//   runPipeline()   the main() loop of sfm.cc:104-129 (fit, freeze-camera solve, filter,
//                   then solve + filter until the point count stops changing).
#pragma once
#include <string>
#include <vector>

#include "../../include/dab.h"
#include "DeepArcManager.hh"

// sfm.cc:31. DENSE_SCHUR-equivalent step (DAB_LINEAR_SOLVER_EXPLICIT_SCHUR); falls back
// to IMPLICIT_SCHUR_PCG when the explicit reduced system does not fit. Prints the
// summary line (the reference prints summary.FullReport()).
void solve(DeepArcManager& deeparcManager, int max_iteration = 1000, int max_second = 3600,
           bool freeze_camera = false);
// Same, with explicit options; fills *summary when non-null. Returns 0 or a DAB_E_* code.
int solveWith(DeepArcManager& m, const dab_options& options, bool freeze_camera, dab_summary* summary);

// Least-squares fit of centre c and squared radius R to the camera centres, from
// c = 0, R = 1, with Ceres' trust-region LM semantics (max_iteration iterations).
// With no centres (non-shared mode, quirk Q6) c and R are left unchanged.
void fitHemisphere(const std::vector<std::vector<double> >& centers, double center[3], double* radius,
                   int max_iteration = 1000);

struct PipelineReport {
  double hemisphere_center[3], hemisphere_radius;
  int rounds, final_blocks, final_points;
  int solves = 0, lm_iterations = 0;  // solve() calls, LM iterations summed over them
  double final_cost = 0.0;            // the last solve's final cost
  double solve_seconds = 0.0, filter_seconds = 0.0, total_seconds = 0.0;
  // breakdown (seconds, summed over the loop): read the .deeparc, hemisphere fit, PLY and
  // output writes, and the DabTimers stages (DabScene.hh)
  double read_seconds = 0.0, fit_seconds = 0.0, write_seconds = 0.0, marshal_seconds = 0.0, setup_seconds = 0.0,
         update_seconds = 0.0, prep_seconds = 0.0, lm_seconds = 0.0, writeback_seconds = 0.0,
         filter_device_seconds = 0.0, filter_host_seconds = 0.0;
};
// sfm.cc main() without the hard-coded paths: reads `input`, writes the outputs whose
// names are non-empty (PLY snapshots are skipped when ply_prefix is empty). verbose: the
// per-iteration progress and the per-solve summary line the reference prints.
PipelineReport runPipeline(const std::string& input, const std::string& output, const std::string& ply_prefix,
                           int max_iteration = 100, int max_second = 3600, double error_boundary = 5.0,
                           bool verbose = true);
