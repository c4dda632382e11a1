// DeepArcManager.cc — .deeparc I/O, PLY export, camera centres and filterPoint3d with the
// reference's semantics (src/DeepArcManager.cc), including its quirks Q1, Q2, Q4, Q6, Q7
// (SURVEY App. C). The residuals behind filterPoint3d come from the GPU (dab_filter).
#include "DeepArcManager.hh"

#include <algorithm>
#include <sched.h>
#include <cctype>
#include <cstdlib>
#include <charconv>
#include <cstdio>
#include <cstring>
#include <thread>
#include <type_traits>
#include <fstream>
#include <iterator>
#include <iostream>
#include <unordered_map>

#include "../csrc/rotation.h"
#include "DabScene.hh"

namespace {

// The reference reads with operator>> and indexes with .at(); a short or inconsistent
// file throws here instead of reading garbage. The file is read whole and parsed from
// memory with std::from_chars (a correctly rounded conversion, so the same doubles as the
// stream's strtod-based extraction) — the stream extraction took ~0.2 s of a ~0.2-s GPU
// pipeline on the 160k-observation config-1 scene. Stream semantics kept: leading white
// space skipped, an optional '+' (from_chars takes only '-'), the longest numeric prefix
// consumed (an int read of "12.5" leaves ".5" for the next read), no inf / nan words.
class Tokens {
 public:
  explicit Tokens(std::string text) : buf_(std::move(text)), p_(buf_.data()), end_(buf_.data() + buf_.size()) {}
  template <class T>
  T take() {
    T v{};
    if (!take_at(p_, end_, v)) throw "Malformed .deeparc file";
    return v;
  }
  // one token from [p, end) into v, p moved past it; false on a malformed token
  template <class T>
  static bool take_at(const char*& p, const char* end, T& v) {
    while (p < end && std::isspace((unsigned char)*p)) ++p;
    const char* q = p;
    if (q < end && *q == '+') ++q;
    if (q >= end || !(std::isdigit((unsigned char)*q) || *q == '-' || *q == '.')) return false;
    if constexpr (std::is_same<T, double>::value) {
      if (fast_double(q, end, v)) {
        p = q;
        return true;
      }
    }
    const auto r = std::from_chars(q, end, v);
    if (r.ec != std::errc()) return false;
    p = r.ptr;
    return true;
  }
  // Decimal -> double without libstdc++'s from_chars (GCC 11: strtod under a per-call locale,
  // ~25 ns a token and serialised across threads). Up to 19 significant digits and a decimal
  // exponent within +-27: the digits and the power of ten are exact in x87 long double (64-bit
  // mantissa), one multiply or divide rounds correctly to it, and the rounding to double is
  // then correct unless the long double sits within one of its ulps of a double half-way
  // point; those, and every other form, go to from_chars. Same value as strtod either way.
  static bool fast_double(const char*& p, const char* end, double& out) {
    static const long double kPow10[28] = {1e0L,  1e1L,  1e2L,  1e3L,  1e4L,  1e5L,  1e6L,  1e7L,  1e8L,  1e9L,
                                           1e10L, 1e11L, 1e12L, 1e13L, 1e14L, 1e15L, 1e16L, 1e17L, 1e18L, 1e19L,
                                           1e20L, 1e21L, 1e22L, 1e23L, 1e24L, 1e25L, 1e26L, 1e27L};
    const char* q = p;
    bool neg = false;
    if (q < end && *q == '-') {
      neg = true;
      ++q;
    }
    unsigned long long m = 0;
    int sig = 0, exp10 = 0;
    bool any = false;
    for (; q < end && *q >= '0' && *q <= '9'; ++q) {
      any = true;
      if (m == 0 && *q == '0') continue;
      if (++sig > 19) return false;
      m = m * 10 + (unsigned)(*q - '0');
    }
    if (q < end && *q == '.') {
      ++q;
      for (; q < end && *q >= '0' && *q <= '9'; ++q) {
        any = true;
        --exp10;
        if (m == 0 && *q == '0') continue;
        if (++sig > 19) return false;
        m = m * 10 + (unsigned)(*q - '0');
      }
    }
    if (!any) return false;
    if (q < end && (*q == 'e' || *q == 'E')) return false;  // exponent forms: from_chars
    if (m == 0) {
      out = neg ? -0.0 : 0.0;
      p = q;
      return true;
    }
    if (exp10 < -27 || exp10 > 27) return false;
    long double v = (long double)m;
    v = exp10 >= 0 ? v * kPow10[exp10] : v / kPow10[-exp10];
    unsigned long long mant;
    std::memcpy(&mant, &v, 8);  // x87 extended: the 64-bit significand (explicit leading bit)
    const unsigned low = (unsigned)(mant & 0x7FF);
    if (low >= 0x3FF && low <= 0x401) return false;  // near a double half-way point
    out = neg ? -(double)v : (double)v;
    p = q;
    return true;
  }
  const char* pos() const { return p_; }
  const char* end() const { return end_; }
  void seek(const char* p) { p_ = p; }

 private:
  std::string buf_;
  const char* p_;
  const char* end_;
};

void fmt6(FILE* f, double v) { std::fprintf(f, "%.6f", v); }  // std::fixed, setprecision(6)
void fmtg(FILE* f, double v) { std::fprintf(f, "%g", v); }    // default ostream format

// The observation section (five tokens per block, one block per line as every writer emits
// it) is most of the file and of its parse time (~25 ns per from_chars double), the point
// section (six tokens per point) the next largest: a section is cut at line starts into
// pieces parsed on several threads into plain arrays (`line(i, p, le)` parses record i from
// one line [p, le)), then the objects are created in file order. A piece whose lines do not
// hold exactly the record's well-formed tokens each, or a section that is not
// line-aligned, is parsed again by the sequential tokenizer (`seq`), which gives the stream
// semantics (tokens may span lines) and the same values.
template <class Line, class Seq>
void parse_section(Tokens& f, int n, int min_parallel, const Line& line, const Seq& seq) {
  const char* p0 = f.pos();
  const char* end = f.end();
  // DAB_READ_THREADS: most parser threads (default: the CPUs this process may run on, at
  // most 16; 1 = sequential)
  static const int tmax = [] {
    if (const char* e = getenv("DAB_READ_THREADS")) return std::max(1, atoi(e));
    int n = (int)std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
    return std::max(1, std::min(n, 16));
  }();
  const int T = n >= min_parallel ? tmax : 1;
  bool parallel_ok = T > 1;
  std::vector<const char*> cut(T + 1, nullptr);
  if (parallel_ok) {
    // the section starts on the line after the previous token: the rest of that line must be blank
    const char* q = static_cast<const char*>(std::memchr(p0, '\n', end - p0));
    parallel_ok = q != nullptr;
    if (parallel_ok) {
      for (const char* c = p0; c < q; ++c) parallel_ok = parallel_ok && std::isspace((unsigned char)*c);
      ++q;
      long long ln = 0;
      int k = 0;
      cut[0] = q;
      for (int t = 1; t <= T && parallel_ok; ++t) {
        const long long want = (long long)n * t / T;
        while (ln < want && q && q < end) {
          q = static_cast<const char*>(std::memchr(q, '\n', end - q));
          if (q) ++q;
          ++ln;
        }
        if (ln < want) parallel_ok = false;
        cut[++k] = q ? q : end;
      }
    }
  }
  std::vector<char> bad(T, 0);
  if (parallel_ok) {
    auto piece = [&](int t) {
      const char* p = cut[t];
      const char* e = cut[t + 1];
      const int i0 = (int)((long long)n * t / T), i1 = (int)((long long)n * (t + 1) / T);
      for (int i = i0; i < i1; ++i) {
        const char* nl = static_cast<const char*>(std::memchr(p, '\n', e - p));
        const char* le = nl ? nl : e;
        if (!line(i, p, le)) {
          bad[t] = 1;
          return;
        }
        while (p < le && std::isspace((unsigned char)*p)) ++p;
        if (p != le) {  // a token too many on the line
          bad[t] = 1;
          return;
        }
        p = nl ? nl + 1 : e;
      }
      if (p != e) bad[t] = 1;
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(piece, t);
    piece(0);
    for (auto& x : th) x.join();
    for (int t = 0; t < T; ++t) parallel_ok = parallel_ok && !bad[t];
    if (parallel_ok) f.seek(cut[T]);
  }
  if (!parallel_ok) {
    f.seek(p0);
    seq();
  }
}

void read_observations(Tokens& f, int n_blocks, std::vector<ParameterBlock*>& params_) {
  std::vector<int> ia(n_blocks), ir(n_blocks), ip(n_blocks);
  std::vector<double> vx(n_blocks), vy(n_blocks);
  parse_section(
      f, n_blocks, 32768,
      [&](int i, const char*& p, const char* le) {
        return Tokens::take_at(p, le, ia[i]) && Tokens::take_at(p, le, ir[i]) && Tokens::take_at(p, le, ip[i]) &&
               Tokens::take_at(p, le, vx[i]) && Tokens::take_at(p, le, vy[i]);
      },
      [&]() {
        for (int i = 0; i < n_blocks; ++i) {
          ia[i] = f.take<int>();
          ir[i] = f.take<int>();
          ip[i] = f.take<int>();
          vx[i] = f.take<double>();
          vy[i] = f.take<double>();
        }
      });
  params_.reserve(params_.size() + n_blocks);
  for (int i = 0; i < n_blocks; ++i) params_.push_back(new ParameterBlock(ia[i], ir[i], ip[i], new Point2d(vx[i], vy[i])));
}

// points: x y z r g b, colour read as double and truncated (Q2)
void read_points(Tokens& f, int n_points, std::vector<Point3d*>& point3d_) {
  std::vector<double> v(6 * (size_t)n_points);
  parse_section(
      f, n_points, 8192,
      [&](int i, const char*& p, const char* le) {
        double* o = &v[6 * (size_t)i];
        for (int j = 0; j < 6; ++j)
          if (!Tokens::take_at(p, le, o[j])) return false;
        return true;
      },
      [&]() {
        for (size_t j = 0; j < v.size(); ++j) v[j] = f.take<double>();
      });
  point3d_.reserve(point3d_.size() + n_points);
  for (int i = 0; i < n_points; ++i) {
    const double* o = &v[6 * (size_t)i];
    point3d_.push_back(new Point3d(o[0], o[1], o[2], (int)o[3], (int)o[4], (int)o[5]));
  }
}

}  // namespace

void Extrinsic::rotationMatrix(double R[9]) { dab::AngleAxisToRotationMatrix(rotation_, R); }

Point3d::~Point3d() {
  for (ParameterBlock* b : blocks_) b->forget_point3d();
}

DeepArcManager::~DeepArcManager() { clear(); }

DabSession& DeepArcManager::dabSession() {
  if (!session_) session_.reset(new DabSession());
  return *session_;
}

void DeepArcManager::clear() {
  // points first: each one clears its blocks' links, so the blocks need not unlink
  for (Point3d* p : point3d_) delete p;
  for (ParameterBlock* b : params_) delete b;
  for (Intrinsic* k : intrinsics_) delete k;
  for (Extrinsic* e : extrinsics_) delete e;
  for (Camera* c : camera_) delete c;
  for (auto& a : hemisphere_)
    for (auto& r : a.second) delete r.second;
  params_.clear();
  point3d_.clear();
  intrinsics_.clear();
  extrinsics_.clear();
  camera_.clear();
  hemisphere_.clear();
}

bool DeepArcManager::read(std::string filename) {
  // DAB_READ_TIMING=1: phase times on stderr
  static const bool timing = getenv("DAB_READ_TIMING") != nullptr;
  double tr = dab_now_seconds();
  auto phase = [&](const char* what) {
    if (!timing) return;
    const double t = dab_now_seconds();
    std::fprintf(stderr, "read %-14s %.2f ms\n", what, 1e3 * (t - tr));
    tr = t;
  };
  std::ifstream in(filename, std::ios::binary);
  if (in.fail()) {
    std::cout << "Cannot read " << filename << std::endl;
    throw "Cannot read input file";
  }
  std::string text;
  in.seekg(0, std::ios::end);
  const std::streamoff size = in.fail() ? -1 : (std::streamoff)in.tellg();
  if (size > 0) {
    text.resize((size_t)size);
    in.seekg(0, std::ios::beg);
    in.read(&text[0], size);
    if (!in) throw "Cannot read input file";
  } else if (size < 0) {
    // not seekable (a pipe, /dev/stdin, a FIFO): read through to EOF
    in.clear();
    text.assign(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
    if (in.bad()) throw "Cannot read input file";
  }
  Tokens f(std::move(text));
  phase("file");
  clear();
  phase("clear");
  ++structure_version_;
  (void)f.take<double>();  // version
  const int n_blocks = f.take<int>(), n_intr = f.take<int>(), n_arc = f.take<int>(), n_ring = f.take<int>(),
            n_points = f.take<int>();
  if (n_blocks < 0 || n_intr < 0 || n_arc < 0 || n_ring < 0 || n_points < 0) throw "Malformed .deeparc file";
  share_extrinsic_ = n_ring != 0;
  arc_size_ = n_arc;
  ring_size_ = n_ring;
  const int n_ext = share_extrinsic_ ? n_arc + n_ring - 1 : n_arc;

  // observation lines: pos_arc pos_ring point_id x y
  read_observations(f, n_blocks, params_);
  phase("observations");
  // intrinsics: cx cy nf f[nf] nk k[nk]; the principal point truncates to int (Q1)
  for (int i = 0; i < n_intr; ++i) {
    Intrinsic* k = new Intrinsic();
    intrinsics_.push_back(k);
    k->id(i);
    const double cx = f.take<double>(), cy = f.take<double>();
    k->center((int)cx, (int)cy);
    double v[2];
    const int nf = f.take<int>();
    if (nf < 0 || nf > 2) throw "Malformed .deeparc file";
    for (int j = 0; j < nf; ++j) v[j] = f.take<double>();
    k->focal(nf, v);
    const int nk = f.take<int>();
    if (nk < 0 || nk > 2) throw "Malformed .deeparc file";
    for (int j = 0; j < nk; ++j) v[j] = f.take<double>();
    k->distrotion(nk, v);
  }
  // extrinsics: tx ty tz nr r[nr]; 3 = angle-axis, 4 = quaternion (w,x,y,z),
  // 9 = column-major rotation matrix (Ceres conventions, DeepArcManager.cc:133-147)
  for (int i = 0; i < n_ext; ++i) {
    Extrinsic* e = new Extrinsic();
    extrinsics_.push_back(e);
    e->id(i);
    const double tx = f.take<double>(), ty = f.take<double>(), tz = f.take<double>();
    e->translation(tx, ty, tz);
    const int nr = f.take<int>();
    if (nr != 3 && nr != 4 && nr != 9) throw "Malformed .deeparc file";
    double rot[9], aa[3];
    for (int j = 0; j < nr; ++j) rot[j] = f.take<double>();
    if (nr == 9) dab::RotationMatrixToAngleAxis(rot, aa);
    else if (nr == 4) dab::QuaternionToAngleAxis(rot, aa);
    e->rotation(nr == 3 ? rot : aa);
  }
  read_points(f, n_points, point3d_);

  phase("cameras, points");
  auto need = [](bool ok) {
    if (!ok) throw "Malformed .deeparc file: index out of range";
  };
  if (share_extrinsic_) {
    // arc a -> extrinsic a (id a); ring r -> extrinsic 0 (r = 0) or n_arc + r - 1 (id r)
    need(n_intr >= n_arc && n_ext >= 1);
    for (int a = 0; a < n_arc; ++a) {
      extrinsics_[a]->id(a);
      for (int r = 0; r < n_ring; ++r) {
        Extrinsic* ring = extrinsics_[ringExtrinsicIndex(r, n_arc)];
        ring->id(r);
        hemisphere_[a][r] = new Camera(intrinsics_[a], extrinsics_[a], ring);
      }
    }
  } else {
    // one camera per distinct extrinsic id, first intrinsic seen (std::map order)
    std::map<int, int> ext_intr;
    for (ParameterBlock* b : params_) ext_intr.insert({b->extrinsic_id(), b->intrinsic_id()});
    for (const auto& ei : ext_intr) {
      need(ei.first >= 0 && ei.first < n_ext && ei.second >= 0 && ei.second < n_intr);
      camera_.push_back(new Camera(intrinsics_[ei.second], extrinsics_[ei.first]));
    }
  }
  {  // every point's link list at its final size (no growth reallocations)
    std::vector<int> nlink(n_points, 0);
    for (ParameterBlock* b : params_) {
      need(b->point3d_id() >= 0 && b->point3d_id() < n_points);
      ++nlink[b->point3d_id()];
    }
    for (int i = 0; i < n_points; ++i) point3d_[i]->reserve_links(nlink[i]);
  }
  for (ParameterBlock* b : params_) {
    need(b->intrinsic_id() >= 0 && b->intrinsic_id() < n_intr);
    b->intrinsic(intrinsics_[b->intrinsic_id()]);
    b->attach_new_point3d(point3d_[b->point3d_id()]);  // a new block: linked once
    if (share_extrinsic_) {
      need(b->pos_arc() < n_ext && b->pos_ring() >= 0 && b->pos_ring() < n_ring);
      b->arc(extrinsics_[b->pos_arc()]);
      b->ring(extrinsics_[ringExtrinsicIndex(b->pos_ring(), n_arc)]);
      b->share_extrinsic(true);
    } else {
      need(b->extrinsic_id() >= 0 && b->extrinsic_id() < n_ext);
      b->extrinsic(extrinsics_[b->extrinsic_id()]);
      b->share_extrinsic(false);
    }
  }
  phase("links");
  return true;
}

std::vector<double> DeepArcManager::cameraPosition(Extrinsic* e) {
  // C = -R^T t
  double R[9];
  e->rotationMatrix(R);
  const double* t = e->translation();
  std::vector<double> c(3);
  for (int i = 0; i < 3; ++i) c[i] = -(R[3 * i] * t[0] + R[3 * i + 1] * t[1] + R[3 * i + 2] * t[2]);
  return c;
}

std::vector<double> DeepArcManager::cameraPosition(Extrinsic* arc, Extrinsic* ring) {
  // P = R_arc (R_ring X + t_ring) + t_arc = 0  =>  C = -R_ring^T t_ring - R_ring^T R_arc^T t_arc
  double Ra[9], Rr[9];
  arc->rotationMatrix(Ra);
  ring->rotationMatrix(Rr);
  const double *ta = arc->translation(), *tr = ring->translation();
  double u[3];  // R_arc^T t_arc (column-major: R^T row i = column i)
  for (int i = 0; i < 3; ++i) u[i] = Ra[3 * i] * ta[0] + Ra[3 * i + 1] * ta[1] + Ra[3 * i + 2] * ta[2];
  std::vector<double> c(3);
  for (int i = 0; i < 3; ++i) {
    const double a = Rr[3 * i] * tr[0] + Rr[3 * i + 1] * tr[1] + Rr[3 * i + 2] * tr[2];
    const double b = Rr[3 * i] * u[0] + Rr[3 * i + 1] * u[1] + Rr[3 * i + 2] * u[2];
    c[i] = -a - b;
  }
  return c;
}

std::vector<std::vector<double> > DeepArcManager::getCameraCenter() {
  std::vector<std::vector<double> > out;
  if (!share_extrinsic_) return out;  // ring_size_ = 0: the arc x ring loop is empty (Q6)
  for (int a = 0; a < arc_size_; ++a)
    for (int r = 0; r < ring_size_; ++r) {
      Camera* cam = hemisphere_[a][r];
      if (r == 0) out.push_back(cameraPosition(cam->arc()));
      else if (a == 0) out.push_back(cameraPosition(cam->ring()));
      else out.push_back(cameraPosition(cam->arc(), cam->ring()));
    }
  return out;
}

void DeepArcManager::writePly(std::string filename) {
  FILE* f = std::fopen(filename.c_str(), "w");
  if (!f) throw "Cannot write output file";
  const int n_cam = share_extrinsic_ ? arc_size_ * ring_size_ : (int)camera_.size();
  std::fprintf(f,
               "ply\nformat ascii 1.0\nelement vertex %d\nproperty float x\nproperty float y\n"
               "property float z\nproperty uchar red\nproperty uchar green\nproperty uchar blue\n"
               "end_header\n",
               (int)point3d_.size() + n_cam);
  auto put = [&](const std::vector<double>& c, const char* colour) {
    for (int i = 0; i < 3; ++i) {
      fmtg(f, c[i]);
      std::fputc(' ', f);
    }
    std::fputs(colour, f);
  };
  if (share_extrinsic_) {
    // arc-only and ring-only cameras green, composed ones magenta
    for (int a = 0; a < arc_size_; ++a)
      for (int r = 0; r < ring_size_; ++r) {
        Camera* cam = hemisphere_[a][r];
        if (r == 0) put(cameraPosition(cam->arc()), "0 255 0\n");
        else if (a == 0) put(cameraPosition(cam->ring()), "0 255 0\n");
        else put(cameraPosition(cam->arc(), cam->ring()), "255 0 255\n");
      }
  } else {
    for (Camera* cam : camera_) put(cameraPosition(cam->extrinsic()), "0 255 0\n");
  }
  for (Point3d* p : point3d_) {
    for (int i = 0; i < 3; ++i) {
      fmtg(f, p->position()[i]);
      std::fputc(' ', f);
    }
    std::fprintf(f, "%d %d %d\n", p->r(), p->g(), p->b());
  }
  std::fclose(f);
}

void DeepArcManager::write(std::string filename) {
  FILE* f = std::fopen(filename.c_str(), "w");
  if (!f) throw "Cannot write output file";
  for (int i = 0; i < (int)point3d_.size(); ++i) point3d_[i]->id(i);  // re-index points
  std::fprintf(f, "0.010000\n%d %d ", (int)params_.size(), (int)intrinsics_.size());
  if (share_extrinsic_) std::fprintf(f, "%d %d ", arc_size_, ring_size_);
  else std::fprintf(f, "%d 0 ", (int)camera_.size());
  std::fprintf(f, "%d\n", (int)point3d_.size());
  for (ParameterBlock* b : params_) {
    const int cam = share_extrinsic_ ? b->ring()->id() : b->extrinsic()->id();
    std::fprintf(f, "%d %d %d ", b->intrinsic()->id(), cam, b->point3d()->id());
    fmt6(f, b->point2d()->x());
    std::fputc(' ', f);
    fmt6(f, b->point2d()->y());
    std::fputc('\n', f);
  }
  for (Intrinsic* k : intrinsics_) {
    fmt6(f, k->center()[0]);
    std::fputc(' ', f);
    fmt6(f, k->center()[1]);
    std::fprintf(f, " %d", k->focal_size());
    for (int j = 0; j < k->focal_size(); ++j) {
      std::fputc(' ', f);
      fmt6(f, k->focal()[j]);
    }
    std::fprintf(f, " %d", k->distrotion_size());
    for (int j = 0; j < k->distrotion_size(); ++j) {
      std::fputc(' ', f);
      fmt6(f, k->distrotion()[j]);
    }
    std::fputc('\n', f);
  }
  for (Extrinsic* e : extrinsics_) {  // always angle-axis (Q7)
    for (int j = 0; j < 3; ++j) {
      fmt6(f, e->translation()[j]);
      std::fputc(' ', f);
    }
    std::fputs("3", f);
    for (int j = 0; j < 3; ++j) {
      std::fputc(' ', f);
      fmt6(f, e->rotation()[j]);
    }
    std::fputc('\n', f);
  }
  for (Point3d* p : point3d_) {
    for (int j = 0; j < 3; ++j) {
      fmt6(f, p->position()[j]);
      std::fputc(' ', f);
    }
    std::fprintf(f, "%d %d %d\n", p->r(), p->g(), p->b());
  }
  std::fclose(f);
}

void DeepArcManager::filterPoint3d(double error_boundary, double* hemisphere_center, double hemisphere_radius) {
  // device: residual per observation, the mse test, the empty-point and hemisphere tests
  std::vector<uint8_t> keep_obs(params_.size(), 1), keep_pt(point3d_.size(), 1);
  if (!params_.empty()) {
    // on the resident problem of the last solve when the structure is unchanged (the
    // residual pass does not depend on the constancy): no set-up, values refreshed only
    DabSession& S = dabSession();
    dab_check(S.ensure(*this, -1));
    const double t0 = dab_now_seconds();
    dab_check(dab_filter(S.handle.h, error_boundary, hemisphere_center, hemisphere_radius, keep_obs.data(),
                         keep_pt.data(), nullptr, nullptr));
    S.t.filter_dev += dab_now_seconds() - t0;
  } else {
    std::fill(keep_pt.begin(), keep_pt.end(), 0);  // no observations: every point is empty
  }
  const double th = dab_now_seconds();
  // host: drop points, then blocks, preserving the survivors' order (std::remove_if). A
  // dropped point clears the links of its blocks (Point3d's destructor), so the blocks
  // dropped with it need no unlink; the filter drops every block of a dropped point.
  size_t w = 0;
  for (size_t i = 0; i < point3d_.size(); ++i) {
    if (keep_pt[i]) point3d_[w++] = point3d_[i];
    else delete point3d_[i];
  }
  const size_t np_old = point3d_.size();
  point3d_.resize(w);
  const size_t np_new = w;
  w = 0;
  for (size_t i = 0; i < params_.size(); ++i) {
    if (keep_obs[i]) params_[w++] = params_[i];
    else delete params_[i];  // unlinks from its point if that one stays
  }
  const bool changed = np_new != np_old || w != keep_obs.size();
  params_.resize(w);
  if (changed) {
    ++structure_version_;  // the resident problem no longer matches
    // the session's arrays follow the same compaction (the next set-up needs no marshal)
    if (session_) session_->filtered(*this, structure_version_ - 1, keep_obs.data(), keep_pt.data());
  }
  // only a session that exists takes the timer: filtering a manager without observations
  // must not create one (that would initialise the GPU on a host-only path)
  if (session_) session_->t.filter_host += dab_now_seconds() - th;
}
