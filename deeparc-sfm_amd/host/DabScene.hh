// DabScene.hh — marshals a DeepArcManager into the SoA dab_problem of include/dab.h and
// writes the solved parameters back into the manager's blocks. It follows the
// observation -> parameter mapping of ParameterBlock::get() (ParameterBlock.hh:68-94)
// and the constancy rules of solve() (sfm.cc:50-63).
#pragma once
#include <vector>

#include "../../include/dab.h"
#include "DeepArcManager.hh"

struct DabScene {
  std::vector<double> xy, points, ext, intr;
  std::vector<int32_t> obs_point, obs_ext0, obs_ext1, obs_intr, intr_nf, intr_nk;
  std::vector<uint8_t> ext_const;
  std::vector<uint8_t> obs_gauge;  // 1: a (0,0) block, whose extrinsic is constant (sfm.cc:50-53)
  dab_problem problem{};

  // Observation o = parameters()->at(o); point ids = index in point3ds(); extrinsic and
  // intrinsic ids = index in extrinsics() / intrinsics(). Throws const char* when a block
  // references a parameter the manager does not own.
  void build(DeepArcManager& m, bool freeze_camera);
  // problem from the arrays as they are (build ends with it)
  void bind(bool freeze_camera);
  // parameter values back into the manager's Point3d / Extrinsic storage
  void write_back(DeepArcManager& m);
  // the manager's current parameter values into points / ext (same structure as build)
  void refresh_values(DeepArcManager& m);
  // the arrays of the manager after filterPoint3d dropped the blocks with keep_obs[o] == 0 and
  // the points with keep_pt[i] == 0 (survivors in order, as the manager compacts its lists):
  // the same arrays build() would make, without walking the blocks
  // false (arrays half-compacted: rebuild) when a kept observation's point was dropped
  bool compact(const uint8_t* keep_obs, const uint8_t* keep_pt);
};

// RAII device handle on the device named by $DAB_DEVICE (default 0).
struct DabHandle {
  dab_handle* h = nullptr;
  DabHandle();
  ~DabHandle();
  DabHandle(const DabHandle&) = delete;
  DabHandle& operator=(const DabHandle&) = delete;
};

// The manager's resident problem: one handle for the manager's lifetime; the problem set
// on it is valid while (version, freeze, sizes) match the manager (DeepArcManager::
// dabSession). ensure() re-marshals and re-sets the problem when they do not, and only
// uploads the parameter values when they do.
// Host-side time of each stage of the sfm.cc loop on this manager, accumulated (seconds):
// marshal = DabScene::build (pointer walk into the SoA arrays), setup = dab_set_problem,
// update = values-only refresh, prep = a solve's table build / graph capture (dab_solve
// wall minus its summary's total time), lm = the LM iterations (summary total time),
// writeback = values back into the manager, filter_dev = dab_filter, filter_host = the
// manager's compaction of blocks and points.
struct DabTimers {
  double marshal = 0, setup = 0, update = 0, prep = 0, lm = 0, writeback = 0, filter_dev = 0, filter_host = 0;
};
double dab_now_seconds();

struct DabSession {
  DabTimers t;
  DabHandle handle;
  DabScene scene;
  bool resident = false;
  bool freeze = false;
  unsigned long long version = 0;
  // the scene's arrays match the manager's structure at scene_version (build, or compact
  // after a filter), so a re-set-up needs no marshal
  bool scene_valid = false;
  unsigned long long scene_version = 0;
  size_t n_blocks = 0, n_points = 0, n_ext = 0, n_intr = 0;
  // freeze < 0: any constancy will do (the filter's residual pass). Returns 0 or a DAB_E_*
  // code; throws const char* when a block references a parameter the manager does not own.
  int ensure(DeepArcManager& m, int freeze);
  // after filterPoint3d: compact the scene instead of rebuilding it (when it was current)
  void filtered(DeepArcManager& m, unsigned long long old_version, const uint8_t* keep_obs, const uint8_t* keep_pt);
};

// throws the library's message as const char* (the reference throws const char*,
// DeepArcManager.cc:30) when rc != 0
void dab_check(int rc);
