// synth.cpp — deterministic synthetic BA problems.
//
// The reference's inputs (data/teabottle_green*.deeparc) are stripped
// (.MISSING_LARGE_BLOBS:1-3), so every benchmark and parity case runs on problems
// generated here with a fixed PRNG (splitmix64 -> xoshiro256**), so this container and
// the GPU box produce bit-identical inputs.
//
//  kind 0, BAL-shaped, non-shared extrinsics (DeepArcManager.cc:58-62): one intrinsic
//    per camera (pos_arc = intrinsic id = camera id, pos_ring = extrinsic id), f=800
//    (|f|=1), |k|=2 radial distortion, pp=(512,512) (integers: Intrinsic.hh:24-27
//    truncates the principal point).
//  kind 1, DeepArc rig, shared extrinsics (DeepArcManager.cc:50-56,166-171): A arcs x
//    R rings; extrinsics 0..A-1 are arcs, ring r>0 is extrinsic A+r-1; camera (a,r)
//    uses arc[a] when r==0, ring[r] when a==0, arc[a]∘ring[r] otherwise
//    (ParameterBlock.hh:75-88). Intrinsic = pos_arc, |f|=2 f=4949.234294,
//    pp=(923,1223), |k|=0 (sample line DeepArcManager.cc:456).
//  The world frame is camera (0,0)'s frame, so arc[0] is the identity (the gauge block,
//  sfm.cc:50-53) and arc[a]∘ring[r] reproduces camera(a,r) exactly.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/dab.h"
#include "dab_internal.h"
#include "rotation.h"

namespace {

struct Rng {
  uint64_t s[4];
  explicit Rng(uint64_t seed) {
    uint64_t x = seed;
    for (int i = 0; i < 4; ++i) {  // splitmix64
      x += 0x9E3779B97F4A7C15ull;
      uint64_t z = x;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      s[i] = z ^ (z >> 31);
    }
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {  // xoshiro256**
    const uint64_t result = rotl(s[1] * 5, 7) * 9;
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return result;
  }
  double uniform() { return (next() >> 11) * 0x1.0p-53; }  // [0,1)
  double uniform(double a, double b) { return a + (b - a) * uniform(); }
  uint32_t below(uint32_t n) { return (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32); }
  double normal() {  // Box–Muller, one value per call (deterministic)
    double u1 = uniform();
    if (u1 < 1e-300) u1 = 1e-300;
    const double u2 = uniform();
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  }
};

struct Pose {
  double R[9];  // row-major here: P = R X + t
  double t[3];
};

void mat_mul(const double A[9], const double B[9], double C[9]) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}
void mat_t(const double A[9], double B[9]) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) B[3 * i + j] = A[3 * j + i];
}
void mat_vec(const double A[9], const double x[3], double y[3]) {
  for (int i = 0; i < 3; ++i) y[i] = A[3 * i] * x[0] + A[3 * i + 1] * x[1] + A[3 * i + 2] * x[2];
}
Pose compose(const Pose& a, const Pose& b) {  // a ∘ b : X -> a(b(X))
  Pose c;
  mat_mul(a.R, b.R, c.R);
  double tb[3];
  mat_vec(a.R, b.t, tb);
  for (int i = 0; i < 3; ++i) c.t[i] = tb[i] + a.t[i];
  return c;
}
Pose inverse(const Pose& a) {
  Pose c;
  mat_t(a.R, c.R);
  double t[3];
  mat_vec(c.R, a.t, t);
  for (int i = 0; i < 3; ++i) c.t[i] = -t[i];
  return c;
}
// camera at centre C looking at the origin; +z forward (projection has no sign flip,
// snavely_reprojection_error.hh:49-50), so visible points have P2 > 0.
Pose look_at(const double C[3]) {
  double f[3] = {-C[0], -C[1], -C[2]};
  const double fn = std::sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
  for (double& v : f) v /= fn;
  double up[3] = {0, 0, 1};
  if (std::fabs(f[2]) > 0.99) { up[0] = 0; up[1] = 1; up[2] = 0; }
  double r[3] = {up[1] * f[2] - up[2] * f[1], up[2] * f[0] - up[0] * f[2], up[0] * f[1] - up[1] * f[0]};
  const double rn = std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  for (double& v : r) v /= rn;
  const double u[3] = {f[1] * r[2] - f[2] * r[1], f[2] * r[0] - f[0] * r[2], f[0] * r[1] - f[1] * r[0]};
  Pose p;
  for (int j = 0; j < 3; ++j) { p.R[j] = r[j]; p.R[3 + j] = u[j]; p.R[6 + j] = f[j]; }
  double RC[3];
  mat_vec(p.R, C, RC);
  for (int i = 0; i < 3; ++i) p.t[i] = -RC[i];
  return p;
}
void pose_to_ext(const Pose& p, double* e) {
  double Rc[9];  // column-major for the Ceres-style converter
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Rc[j * 3 + i] = p.R[3 * i + j];
  dab::RotationMatrixToAngleAxis(Rc, e);
  e[3] = p.t[0]; e[4] = p.t[1]; e[5] = p.t[2];
}
void ball_point(Rng& g, double radius, double X[3]) {
  for (;;) {
    const double x = g.uniform(-1, 1), y = g.uniform(-1, 1), z = g.uniform(-1, 1);
    if (x * x + y * y + z * z <= 1.0) { X[0] = radius * x; X[1] = radius * y; X[2] = radius * z; return; }
  }
}

bool sizes_of(const dab_synth_config* c, int32_t* no, int32_t* np, int32_t* ne, int32_t* ni) {
  if (!c || c->num_points < 0 || c->obs_per_point < 1) return false;
  if (c->kind == 0) {
    if (c->num_cameras < 1 || c->obs_per_point > c->num_cameras) return false;
    *ne = c->num_cameras;
    *ni = c->num_cameras;
  } else if (c->kind == 1) {
    if (c->num_arcs < 1 || c->num_rings < 1) return false;
    if (c->obs_per_point > c->num_arcs * c->num_rings) return false;
    *ne = c->num_rings > 0 ? c->num_arcs + c->num_rings - 1 : c->num_arcs;
    *ni = c->num_arcs;
  } else {
    return false;
  }
  const int64_t nobs = (int64_t)c->num_points * c->obs_per_point;
  if (nobs > INT32_MAX) return false;
  *no = (int32_t)nobs;
  *np = c->num_points;
  return true;
}

}  // namespace

extern "C" int dab_synth_sizes(const dab_synth_config* cfg, int32_t* num_obs, int32_t* num_points,
                               int32_t* num_ext, int32_t* num_intr) {
  int32_t no, np, ne, ni;
  if (!sizes_of(cfg, &no, &np, &ne, &ni)) return dab::set_error(DAB_E_INVALID, "dab_synth_sizes: bad config");
  if (num_obs) *num_obs = no;
  if (num_points) *num_points = np;
  if (num_ext) *num_ext = ne;
  if (num_intr) *num_intr = ni;
  return DAB_OK;
}

extern "C" int dab_synth_fill(const dab_synth_config* cfg, dab_problem* p, uint8_t* ext_const) {
  int32_t no, np, ne, ni;
  if (!sizes_of(cfg, &no, &np, &ne, &ni)) return dab::set_error(DAB_E_INVALID, "dab_synth_fill: bad config");
  if (!p || p->num_obs != no || p->num_points != np || p->num_ext != ne || p->num_intr != ni)
    return dab::set_error(DAB_E_INVALID, "dab_synth_fill: problem sizes do not match dab_synth_sizes");
  if (!p->obs_xy || !p->obs_point || !p->obs_ext0 || !p->obs_ext1 || !p->obs_intr || !p->points ||
      !p->ext || !p->intr || !p->intr_nf || !p->intr_nk)
    return dab::set_error(DAB_E_INVALID, "dab_synth_fill: null array");
  double* obs_xy = const_cast<double*>(p->obs_xy);
  int32_t* obs_point = const_cast<int32_t*>(p->obs_point);
  int32_t* obs_ext0 = const_cast<int32_t*>(p->obs_ext0);
  int32_t* obs_ext1 = const_cast<int32_t*>(p->obs_ext1);
  int32_t* obs_intr = const_cast<int32_t*>(p->obs_intr);
  double* intr = const_cast<double*>(p->intr);
  int32_t* nf = const_cast<int32_t*>(p->intr_nf);
  int32_t* nk = const_cast<int32_t*>(p->intr_nk);
  Rng g(cfg->seed ? cfg->seed : 1);

  const int ncam = cfg->kind == 0 ? cfg->num_cameras : cfg->num_arcs * cfg->num_rings;
  std::vector<Pose> cam(ncam);       // true pose of each physical camera (world -> cam)
  std::vector<int32_t> cam_e0(ncam), cam_e1(ncam), cam_intr(ncam);
  std::vector<uint8_t> cam_is00(ncam, 0);
  std::vector<Pose> ext_true(ne);
  Pose obj_to_world;

  if (cfg->kind == 0) {
    for (int c = 0; c < ncam; ++c) {
      double C[3];
      for (;;) {  // uniform on the upper hemisphere, radius 1, away from the pole/horizon
        double d[3] = {g.normal(), g.normal(), g.normal()};
        const double n = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
        for (double& v : d) v /= n;
        if (d[2] > 0.15 && d[2] < 0.95) { C[0] = d[0]; C[1] = d[1]; C[2] = d[2]; break; }
      }
      cam[c] = look_at(C);
      ext_true[c] = cam[c];
      cam_e0[c] = c;
      cam_e1[c] = -1;
      cam_intr[c] = c;
      cam_is00[c] = c == 0;  // (pos_arc, pos_ring) = (intrinsic 0, extrinsic 0)
      double* K = intr + 6 * (size_t)c;
      K[0] = 512; K[1] = 512; K[2] = 800; K[3] = 800;
      K[4] = g.uniform(-0.1, 0.1);
      K[5] = g.uniform(-0.01, 0.01);
      nf[c] = 1;
      nk[c] = 2;
    }
  } else {
    const int A = cfg->num_arcs, R = cfg->num_rings;
    std::vector<Pose> phys(A);
    for (int a = 0; a < A; ++a) {  // arc cameras: elevation 10..80 deg, azimuth 0
      const double el = (10.0 + (A > 1 ? 70.0 * a / (A - 1) : 0.0)) * M_PI / 180.0;
      const double C[3] = {std::cos(el), 0.0, std::sin(el)};
      phys[a] = look_at(C);
    }
    const Pose cam0 = phys[0], cam0_inv = inverse(phys[0]);
    obj_to_world = cam0;
    for (int a = 0; a < A; ++a) ext_true[a] = compose(phys[a], cam0_inv);  // arc[0] = I
    for (int r = 1; r < R; ++r) {  // turntable about z, expressed in camera-0's frame
      const double ang = 2.0 * M_PI * r / R, c = std::cos(ang), s = std::sin(ang);
      Pose rot;
      const double Rz[9] = {c, -s, 0, s, c, 0, 0, 0, 1};
      std::memcpy(rot.R, Rz, sizeof(Rz));
      rot.t[0] = rot.t[1] = rot.t[2] = 0;
      ext_true[A + r - 1] = compose(cam0, compose(rot, cam0_inv));
    }
    for (int a = 0; a < A; ++a)
      for (int r = 0; r < R; ++r) {
        const int c = a * R + r;
        if (r == 0) { cam_e0[c] = a; cam_e1[c] = -1; }
        else if (a == 0) { cam_e0[c] = A + r - 1; cam_e1[c] = -1; }
        else { cam_e0[c] = a; cam_e1[c] = A + r - 1; }
        cam[c] = cam_e1[c] >= 0 ? compose(ext_true[cam_e0[c]], ext_true[cam_e1[c]]) : ext_true[cam_e0[c]];
        cam_intr[c] = a;
        cam_is00[c] = (a == 0 && r == 0);
      }
    for (int a = 0; a < A; ++a) {
      double* K = intr + 6 * (size_t)a;
      K[0] = 923; K[1] = 1223; K[2] = 4949.234294; K[3] = 4949.234294; K[4] = 0; K[5] = 0;
      nf[a] = 2;
      nk[a] = 0;
    }
  }

  // initial extrinsics = truth + noise, drawn from the camera stream so that every shard
  // of one global problem gets identical cameras (the gauge extrinsic 0 stays exact)
  for (int e = 0; e < ne; ++e) {
    double* E = p->ext + 6 * (size_t)e;
    pose_to_ext(ext_true[e], E);
    if (cfg->kind == 1 && e == 0) { E[0] = E[1] = E[2] = E[3] = E[4] = E[5] = 0.0; }
    if (e == 0) continue;
    for (int k = 0; k < 3; ++k) E[k] += cfg->rot_noise * g.normal();
    for (int k = 3; k < 6; ++k) E[k] += cfg->trans_noise * g.normal();
  }
  if (cfg->point_seed) g = Rng(cfg->point_seed);

  // true points (object frame for the rig is mapped into camera-0's frame)
  std::vector<double> Xtrue(3 * (size_t)np);
  for (int i = 0; i < np; ++i) {
    double X[3];
    ball_point(g, 0.3, X);
    if (cfg->kind == 1) {  // object (turntable) frame -> world = camera-(0,0) frame
      double Y[3];
      mat_vec(obj_to_world.R, X, Y);
      for (int k = 0; k < 3; ++k) X[k] = Y[k] + obj_to_world.t[k];
    }
    for (int k = 0; k < 3; ++k) Xtrue[3 * (size_t)i + k] = X[k];
  }

  // observations: each point seen by m distinct random cameras
  const int m = cfg->obs_per_point;
  std::vector<int32_t> pick(m);
  bool any00 = false;
  size_t o = 0;
  for (int i = 0; i < np; ++i) {
    for (int k = 0; k < m; ++k) {
      for (;;) {
        const int32_t c = (int32_t)g.below((uint32_t)ncam);
        bool dup = false;
        for (int q = 0; q < k; ++q) dup |= pick[q] == c;
        if (!dup) { pick[k] = c; break; }
      }
    }
    for (int k = 0; k < m; ++k, ++o) {
      const int c = pick[k];
      double P[3];
      mat_vec(cam[c].R, &Xtrue[3 * (size_t)i], P);
      for (int q = 0; q < 3; ++q) P[q] += cam[c].t[q];
      const double* K = intr + 6 * (size_t)cam_intr[c];
      const int ii = cam_intr[c];
      const double xp = P[0] / P[2], yp = P[1] / P[2];
      const double r2 = xp * xp + yp * yp;
      double d = 1.0;
      if (nk[ii] == 2) d = 1.0 + r2 * (K[4] + K[5] * r2);
      if (nk[ii] == 1) d = 1.0 + r2 * K[4];
      const double fy = nf[ii] == 2 ? K[3] : K[2];
      obs_xy[2 * o] = K[2] * d * xp + K[0] + cfg->pixel_noise * g.normal();
      obs_xy[2 * o + 1] = fy * d * yp + K[1] + cfg->pixel_noise * g.normal();
      obs_point[o] = i;
      obs_ext0[o] = cam_e0[c];
      obs_ext1[o] = cam_e1[c];
      obs_intr[o] = cam_intr[c];
      any00 |= cam_is00[c] != 0;
    }
  }
  // deterministic shuffle of the observation order (the library must not rely on it)
  for (size_t i = (size_t)no; i > 1; --i) {
    const size_t j = (size_t)g.below((uint32_t)i);
    const size_t a = i - 1;
    std::swap(obs_xy[2 * a], obs_xy[2 * j]);
    std::swap(obs_xy[2 * a + 1], obs_xy[2 * j + 1]);
    std::swap(obs_point[a], obs_point[j]);
    std::swap(obs_ext0[a], obs_ext0[j]);
    std::swap(obs_ext1[a], obs_ext1[j]);
    std::swap(obs_intr[a], obs_intr[j]);
  }

  // initial points = truth + noise
  for (int i = 0; i < np; ++i)
    for (int k = 0; k < 3; ++k)
      p->points[3 * (size_t)i + k] = Xtrue[3 * (size_t)i + k] + cfg->point_noise * g.normal();
  if (ext_const) {
    std::memset(ext_const, 0, (size_t)ne);
    if (any00) ext_const[0] = 1;  // sfm.cc:50-53
  }
  p->freeze_camera = 0;
  return DAB_OK;
}
