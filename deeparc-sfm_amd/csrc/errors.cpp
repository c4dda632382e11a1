// errors.cpp — thread-local error state behind dab_last_error().
#include <cstring>
#include <string>

#include "dab_internal.h"

namespace {
thread_local std::string g_last_error;
}

namespace dab {
int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
void clear_error() { g_last_error.clear(); }
}  // namespace dab

extern "C" const char* dab_last_error(void) { return g_last_error.c_str(); }
extern "C" int dab_abi_version(void) { return DAB_ABI_VERSION; }

extern "C" void dab_options_init(dab_options* o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  // ceres::Solver::Options defaults + the values set at sfm.cc:66-71
  o->max_num_iterations = 50;  // Ceres default; the reference passes 100 (sfm.cc:111,121)
  o->linear_solver_type = DAB_LINEAR_SOLVER_EXPLICIT_SCHUR;  // DENSE_SCHUR, sfm.cc:67
  o->max_solver_time_in_seconds = 1e6;
  o->function_tolerance = 1e-6;
  o->gradient_tolerance = 1e-10;
  o->parameter_tolerance = 1e-8;
  o->min_relative_decrease = 1e-3;
  o->initial_trust_region_radius = 1e4;
  o->max_trust_region_radius = 1e16;
  o->min_trust_region_radius = 1e-32;
  o->min_lm_diagonal = 1e-6;
  o->max_lm_diagonal = 1e32;
  o->max_num_consecutive_invalid_steps = 5;
  o->jacobi_scaling = 1;
  o->minimizer_progress_to_stdout = 0;
  o->num_threads = 16;  // sfm.cc:9,70 (CPU paths only)
  o->max_linear_solver_iterations = 500;
  o->min_linear_solver_iterations = 0;
  o->eta = 1e-1;
  o->pcg_fp32 = 0;
}
