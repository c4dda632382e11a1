// DeepArcManager.hh — host-side scene container with the reference's public interface
// (src/DeepArcManager.hh): .deeparc reader/writer, PLY export, camera centres and
// filterPoint3d. The numeric work behind filterPoint3d (a residual per observation) runs
// on the GPU through libdab (dab_filter); the object-graph edits stay on the host, in
// the reference's order, so the surviving blocks and points are the reference's.
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "Geometry.hh"
#include "ParameterBlock.hh"

struct DabSession;  // DabScene.hh: the manager's resident libdab problem (handle reuse)

class DeepArcManager {
 public:
  DeepArcManager() = default;
  ~DeepArcManager();
  DeepArcManager(const DeepArcManager&) = delete;
  DeepArcManager& operator=(const DeepArcManager&) = delete;

  bool isShareExtrinsic() { return share_extrinsic_; }
  // DeepArcManager.cc:26-74. Throws const char* when the file cannot be read.
  bool read(std::string filename);
  // DeepArcManager.cc:263-328 (cameras first, then points; default stream format).
  void writePly(std::string filename);
  std::vector<ParameterBlock*>* parameters() { return &params_; }
  std::vector<Point3d*>* point3ds() { return &point3d_; }
  // DeepArcManager.cc:332-424 (quirk Q4: drops observations with mse < error_boundary).
  void filterPoint3d(double error_boundary, double* hemisphere_center, double hemisphere_radius);
  // DeepArcManager.cc:426-499 (std::fixed, 6 decimals, angle-axis rotations; quirk Q7).
  void write(std::string filename);
  // DeepArcManager.cc:501-518: arc x ring camera centres (empty in non-shared mode, Q6).
  std::vector<std::vector<double> > getCameraCenter();

  // accessors the reference keeps private, needed by the solver adapter
  std::vector<Intrinsic*>* intrinsics() { return &intrinsics_; }
  std::vector<Extrinsic*>* extrinsics() { return &extrinsics_; }
  int arcSize() const { return arc_size_; }
  int ringSize() const { return ring_size_; }
  // One libdab handle per manager, kept across solve() / filterPoint3d() (the sfm.cc loop,
  // sfm.cc:104-129): the problem stays resident on the device while the manager's
  // structure is unchanged, so a filter after a solve, or a solve of unchanged structure,
  // only refreshes the parameter values. structureVersion() changes whenever read() or
  // filterPoint3d() change the blocks or points.
  DabSession& dabSession();
  unsigned long long structureVersion() const { return structure_version_; }

 private:
  std::unique_ptr<DabSession> session_;
  unsigned long long structure_version_ = 0;
  int arc_size_ = 0, ring_size_ = 0;
  bool share_extrinsic_ = false;
  std::map<int, std::map<int, Camera*> > hemisphere_;
  std::vector<Intrinsic*> intrinsics_;
  std::vector<Extrinsic*> extrinsics_;
  std::vector<Camera*> camera_;
  std::vector<ParameterBlock*> params_;
  std::vector<Point3d*> point3d_;

  void clear();
  static int ringExtrinsicIndex(int ring_position, int arc_size) {
    return ring_position == 0 ? 0 : ring_position + arc_size - 1;
  }
  std::vector<double> cameraPosition(Extrinsic* e);
  std::vector<double> cameraPosition(Extrinsic* arc, Extrinsic* ring);
};
