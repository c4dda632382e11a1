// Geometry.hh — the reference's parameter containers (src/Point/*.hh, src/Camera/*.hh)
// with the same public accessors, so host code written against the reference compiles
// against this library. Storage layout matches the reference: every block is a small
// double array that the solver writes back in place (sfm.cc:47-48 semantics).
#pragma once
#include <algorithm>
#include <mutex>
#include <set>
#include <vector>

class ParameterBlock;

// Fixed-size object pool behind a class's operator new / delete: the reader allocates one
// ParameterBlock and one Point2d per observation (320k objects for the 160k-observation
// config-1 scene) and the filter and the manager's destructor delete them one by one. Each
// thread keeps its own free list and trades nodes with the process-wide list (64K-object
// chunks, kept for the life of the process) in batches of kBatch under a mutex, so a take or
// a give is a few instructions and no lock. An object may be freed on another thread than
// the one that made it.
template <size_t SIZE>
class ObjectPool {
 public:
  static void* take() {
    Local& l = local();
    if (!l.head) l.refill();
    Node* n = l.head;
    l.head = n->next;
    --l.count;
    return n;
  }
  static void give(void* p) {
    if (!p) return;
    Local& l = local();
    Node* n = static_cast<Node*>(p);
    n->next = l.head;
    l.head = n;
    if (++l.count >= 2 * kBatch) l.flush(kBatch);
  }

 private:
  union Node {
    Node* next;
    alignas(16) unsigned char bytes[SIZE];
  };
  static constexpr size_t kChunk = 1 << 16, kBatch = 4096;
  struct Global {
    std::mutex mu;
    Node* head = nullptr;
  };
  static Global& global() {
    static Global* g = new Global();  // never destroyed: thread-local flushes may run at exit
    return *g;
  }
  struct Local {
    Node* head = nullptr;
    size_t count = 0;
    void refill() {
      Global& g = global();
      std::lock_guard<std::mutex> lk(g.mu);
      if (!g.head) {
        Node* c = static_cast<Node*>(::operator new(sizeof(Node) * kChunk));
        for (size_t i = 0; i + 1 < kChunk; ++i) c[i].next = &c[i + 1];
        c[kChunk - 1].next = nullptr;
        g.head = c;
      }
      // up to kBatch nodes from the global list
      Node* first = g.head;
      Node* last = first;
      size_t n = 1;
      while (n < kBatch && last->next) {
        last = last->next;
        ++n;
      }
      g.head = last->next;
      last->next = head;
      head = first;
      count += n;
    }
    // the nodes past the first `keep` back to the global list
    void flush(size_t keep) {
      Node* cut = head;
      Node** link = &head;
      for (size_t i = 0; i < keep && cut; ++i) {
        link = &cut->next;
        cut = cut->next;
      }
      if (!cut) return;
      Node* last = cut;
      size_t n = 1;
      while (last->next) {
        last = last->next;
        ++n;
      }
      *link = nullptr;
      count -= n;
      Global& g = global();
      std::lock_guard<std::mutex> lk(g.mu);
      last->next = g.head;
      g.head = cut;
    }
    ~Local() { flush(0); }
  };
  static Local& local() {
    thread_local Local l;
    return l;
  }
};
#define DAB_POOLED(T)                                                              \
  static void* operator new(size_t n) {                                            \
    return n == sizeof(T) ? ObjectPool<sizeof(T)>::take() : ::operator new(n);    \
  }                                                                                \
  static void operator delete(void* p, size_t n) {                                 \
    if (n == sizeof(T)) ObjectPool<sizeof(T)>::give(p);                            \
    else ::operator delete(p);                                                     \
  }

// Point/Point2d.hh
class Point2d {
 public:
  DAB_POOLED(Point2d)
  Point2d(double x, double y) : x_(x), y_(y) {}
  double x() { return x_; }
  double y() { return y_; }

 private:
  double x_, y_;
};

// Point/Point3d.hh. Colour is stored as int: the loader reads doubles and truncates
// (quirk Q2, DeepArcManager.cc:155-160).
class Point3d {
 public:
  Point3d(double x, double y, double z, int r = 255, int g = 255, int b = 255)
      : require_remove_(false), r_(r), g_(g), b_(b), id_(-1), position_{x, y, z} {}
  // the blocks still linked to this point forget it (ParameterBlock::point3d() becomes null),
  // so deleting the points before their blocks needs no per-block unlink (DeepArcManager.cc)
  ~Point3d();
  Point3d(const Point3d&) = delete;
  Point3d& operator=(const Point3d&) = delete;
  int r() { return r_; }
  int g() { return g_; }
  int b() { return b_; }
  int id() { return id_; }
  void id(int v) { id_ = v; }
  double* position() { return position_; }
  void require_remove(bool v) { require_remove_ = v; }
  bool require_remove() { return require_remove_; }
  // observation links (ParameterBlock::point3d keeps them current). Held as a small
  // vector (a point has a handful of observations; the set's node allocations were most
  // of the reader's time on 160k observations); total_link() still returns the
  // reference's std::set.
  void link(ParameterBlock* b) {
    if (std::find(blocks_.begin(), blocks_.end(), b) == blocks_.end()) blocks_.push_back(b);
  }
  void unlink(ParameterBlock* b) {
    auto it = std::find(blocks_.begin(), blocks_.end(), b);
    if (it != blocks_.end()) {
      *it = blocks_.back();
      blocks_.pop_back();
    }
  }
  std::set<ParameterBlock*> total_link() { return std::set<ParameterBlock*>(blocks_.begin(), blocks_.end()); }
  void reserve_links(size_t n) { blocks_.reserve(n); }
  // a block that is linked for the first time (the reader): no duplicate search
  void link_new(ParameterBlock* b) { blocks_.push_back(b); }
  bool empty() { return blocks_.empty(); }
  // the solver adapter's scratch: this point's index in the manager's list (DabScene::build)
  int slot() { return slot_; }
  void slot(int v) { slot_ = v; }

 private:
  int slot_ = -1;
  bool require_remove_;
  int r_, g_, b_, id_;
  double position_[3];
  std::vector<ParameterBlock*> blocks_;
};

// Camera/Intrinsic.hh. center() takes ints: the principal point is truncated on load
// (quirk Q1, Intrinsic.hh:24-27).
class Intrinsic {
 public:
  double* focal() { return focal_; }
  double* center() { return center_; }
  double* distrotion() { return distortion_; }
  int focal_size() { return focal_size_; }
  int distrotion_size() { return distortion_size_; }
  int id() { return id_; }
  void id(int v) { id_ = v; }
  void focal(int n, const double* f) {
    focal_size_ = n;
    std::copy(f, f + n, focal_);
  }
  void distrotion(int n, const double* k) {
    distortion_size_ = n;
    std::copy(k, k + n, distortion_);
  }
  void center(int cx, int cy) {
    center_[0] = cx;
    center_[1] = cy;
  }
  int slot() { return slot_; }  // adapter scratch (DabScene::build)
  void slot(int v) { slot_ = v; }

 private:
  int slot_ = -1;
  double focal_[2] = {0, 0}, center_[2] = {0, 0}, distortion_[2] = {0, 0};
  int focal_size_ = 0, distortion_size_ = 0, id_ = -1;
};

// Camera/Extrinsic.hh: angle-axis rotation + translation, P = R(w) X + t.
class Extrinsic {
 public:
  double* rotation() { return rotation_; }
  double* translation() { return translation_; }
  int id() { return id_; }
  void id(int v) { id_ = v; }
  void rotation(const double* w) { std::copy(w, w + 3, rotation_); }
  void translation(double x, double y, double z) {
    translation_[0] = x;
    translation_[1] = y;
    translation_[2] = z;
  }
  // R(w) column-major (ceres::AngleAxisToRotationMatrix, Extrinsic.hh:12-17)
  void rotationMatrix(double R[9]);
  int slot() { return slot_; }  // adapter scratch (DabScene::build)
  void slot(int v) { slot_ = v; }

 private:
  int slot_ = -1;
  double rotation_[3] = {0, 0, 0}, translation_[3] = {0, 0, 0};
  int id_ = -1;
};

// Camera/Camera.hh
class Camera {
 public:
  Camera(Intrinsic* k, Extrinsic* e) : intrinsic_(k), extrinsic_(e) {}
  Camera(Intrinsic* k, Extrinsic* arc, Extrinsic* ring) : intrinsic_(k), arc_(arc), ring_(ring) {}
  Intrinsic* intrinsic() { return intrinsic_; }
  Extrinsic* extrinsic() { return extrinsic_; }
  Extrinsic* arc() { return arc_; }
  Extrinsic* ring() { return ring_; }

 private:
  Intrinsic* intrinsic_ = nullptr;
  Extrinsic *extrinsic_ = nullptr, *arc_ = nullptr, *ring_ = nullptr;
};
