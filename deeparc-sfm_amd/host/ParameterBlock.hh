// ParameterBlock.hh — one observation and the parameter blocks its residual reads
// (reference src/ParameterBlock.hh, same accessors). In shared-extrinsic (rig) mode the
// camera is the composition arc∘ring unless pos_arc or pos_ring is 0
// (ParameterBlock.hh:24-28, 68-94).
#pragma once
#include <vector>

#include "Geometry.hh"

class ParameterBlock {
 public:
  DAB_POOLED(ParameterBlock)
  ParameterBlock(int position_arc, int position_ring, int point3d_id, Point2d* point2d)
      : pos_arc_(position_arc), pos_ring_(position_ring), point3d_id_(point3d_id), point2d_(point2d) {}
  ~ParameterBlock() {
    if (point3d_) point3d_->unlink(this);
    delete point2d_;
  }
  ParameterBlock(const ParameterBlock&) = delete;
  ParameterBlock& operator=(const ParameterBlock&) = delete;

  Extrinsic* arc() { return arc_; }
  Extrinsic* ring() { return ring_; }
  Extrinsic* extrinsic() { return extrinsic_; }
  Point2d* point2d() { return point2d_; }
  Point3d* point3d() { return point3d_; }
  Intrinsic* intrinsic() { return intrinsic_; }
  // non-shared mode: pos_arc is the intrinsic id, pos_ring the extrinsic id
  int intrinsic_id() { return pos_arc_; }
  int extrinsic_id() { return pos_ring_; }
  int point3d_id() { return point3d_id_; }
  int pos_arc() { return pos_arc_; }
  int pos_ring() { return pos_ring_; }
  bool share_extrinsic() { return share_extrinsic_; }
  bool require_remove() { return require_remove_; }
  bool compose_extrinsic() { return share_extrinsic_ && pos_arc_ != 0 && pos_ring_ != 0; }

  void arc(Extrinsic* e) { arc_ = e; }
  void ring(Extrinsic* e) { ring_ = e; }
  void extrinsic(Extrinsic* e) { extrinsic_ = e; }
  void point2d(Point2d* p) { point2d_ = p; }
  void intrinsic(Intrinsic* k) { intrinsic_ = k; }
  void point3d(Point3d* p) {
    if (point3d_) point3d_->unlink(this);
    point3d_ = p;
    if (point3d_) point3d_->link(this);
  }
  // the reader's first link of a new block (point3d() == nullptr before)
  void attach_new_point3d(Point3d* p) {
    point3d_ = p;
    p->link_new(this);
  }
  // the linked point is going away (Point3d's destructor): forget it without unlinking
  void forget_point3d() { point3d_ = nullptr; }
  void share_extrinsic(bool v) { share_extrinsic_ = v; }
  void require_remove(bool v) { require_remove_ = v; }

  // The extrinsic(s) the residual uses: (first, second-or-null). Ceres-side this is the
  // tail of get(); the solver adapter reads it to build the gather indices.
  Extrinsic* first_extrinsic() {
    if (!share_extrinsic_) return extrinsic_;
    if (pos_ring_ == 0) return arc_;    // (0,0) and (a,0): the arc camera
    if (pos_arc_ == 0) return ring_;    // (0,r): the ring camera
    return arc_;                        // (a,r): arc ∘ ring
  }
  Extrinsic* second_extrinsic() { return compose_extrinsic() ? ring_ : nullptr; }

  // Parameter pointers in the reference's order: X, pp, focal, distortion, then w,t
  // (and w_ring, t_ring when composed).
  std::vector<double*> get() {
    std::vector<double*> out{point3d_->position(), intrinsic_->center(), intrinsic_->focal(),
                             intrinsic_->distrotion()};
    Extrinsic* e0 = first_extrinsic();
    out.push_back(e0->rotation());
    out.push_back(e0->translation());
    if (Extrinsic* e1 = second_extrinsic()) {
      out.push_back(e1->rotation());
      out.push_back(e1->translation());
    }
    return out;
  }

 private:
  bool share_extrinsic_ = false, require_remove_ = false;
  int pos_arc_, pos_ring_, point3d_id_;
  Point2d* point2d_;
  Intrinsic* intrinsic_ = nullptr;
  Extrinsic *extrinsic_ = nullptr, *arc_ = nullptr, *ring_ = nullptr;
  Point3d* point3d_ = nullptr;
};
