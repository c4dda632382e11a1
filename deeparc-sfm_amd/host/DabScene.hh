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
  dab_problem problem{};

  // Observation o = parameters()->at(o); point ids = index in point3ds(); extrinsic and
  // intrinsic ids = index in extrinsics() / intrinsics(). Throws const char* when a block
  // references a parameter the manager does not own.
  void build(DeepArcManager& m, bool freeze_camera);
  // parameter values back into the manager's Point3d / Extrinsic storage
  void write_back(DeepArcManager& m);
};

// RAII device handle on the device named by $DAB_DEVICE (default 0).
struct DabHandle {
  dab_handle* h = nullptr;
  DabHandle();
  ~DabHandle();
  DabHandle(const DabHandle&) = delete;
  DabHandle& operator=(const DabHandle&) = delete;
};

// throws the library's message as const char* (the reference throws const char*,
// DeepArcManager.cc:30) when rc != 0
void dab_check(int rc);
