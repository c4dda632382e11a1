// dab_pcg.hip — implicit-Schur preconditioned conjugate gradients on the reduced camera
// system (DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG; SURVEY §8a row a7, "Schur + PCG").
//
// S = (s U s + D^2 + cross) - sum_p Y_p Y_p^T is never formed. One matrix-vector product
// S v is two streaming passes over the camera-major Y records (144 B / entry):
//   point pass   t_p = sum_{e in p} Y_e^T v_cam(e)            (gathers Y_e by position)
//   camera pass  w_c = -sum_{pos in c} Y_pos t_pt(pos)         (contiguous records, chunked)
// followed, after the cross-rank all-reduce of w, by one work-group that adds the camera
// block diagonal / arc∘ring cross terms and runs the CG scalar recurrences. The
// preconditioner is block Jacobi on S (Ceres' SCHUR_JACOBI): M_c = diag block of S.
//
// The recurrences follow Ceres' ConjugateGradientsSolver (conjugate_gradients_solver.h,
// external, Ceres 2.x; restated, not verified in this container): x0 = 0, r = b,
// z = M^-1 r, rho = r.z, p = z + (rho / rho_prev) p, q = S p, alpha = rho / p.q,
// x += alpha p, r -= alpha q (r = b - S x every 10th iteration), Q1 = -x.(b + r),
// stop when iter * (Q1 - Q0) / Q1 < eta (Nash & Sofer; eta = Solver::Options::eta) or at
// max_num_iterations; p.q <= 0 stops with the current x; rho, beta or alpha zero/inf is a
// linear solver failure (the LM step is then invalid).
//
// All CG control lives on the device (PcgState) so the host enqueues iterations in batches
// without a round trip; every kernel returns at once after the state leaves "running".
// Every reduction has a fixed order, so results are bitwise reproducible and identical on
// every rank.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include <cfloat>

#include "dab_kernels.h"
#include "dab_wave.h"

namespace dab {

namespace {

constexpr int kOneWG = 1024;

__device__ __forceinline__ double wg_sum(double v, double* sh) {
  // fixed-order sum over a 1024-thread work-group, result broadcast to every thread
  v = wave_sum_lane63(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 63) sh[w] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i];
  return t;
}

__device__ __forceinline__ bool zero_or_inf(double x) { return x == 0.0 || isinf(x); }

// upper-packed index of (a, b), a <= b, in a symmetric 6x6
__device__ __forceinline__ int up6(int a, int b) { return a * 6 - (a * (a - 1)) / 2 + (b - a); }

}  // namespace

// ---- setup ---------------------------------------------------------------------------

// per chunk of camera-major positions: 21 upper entries of sum Z Z^T over same-point runs
// (the exact diagonal S block) | 6 of -sum Y q_p
template <class YT>
__global__ __launch_bounds__(256) void k_pcg_diag_rhs_partial(DevView v, const int* __restrict__ chunk_beg,
                                                              const int* __restrict__ run,
                                                              const YT* __restrict__ Y,
                                                              const double* __restrict__ q,
                                                              double* __restrict__ partial) {
  const int c = blockIdx.x;
  const int b = chunk_beg[c], e = chunk_beg[c + 1];
  double acc[27];
#pragma unroll
  for (int i = 0; i < 27; ++i) acc[i] = 0.0;
  for (int i = b + threadIdx.x; i < e; i += blockDim.x) {
    const int p = v.cm_pt[i];
    const double2 qa = reinterpret_cast<const double2*>(q)[2 * (size_t)p];
    const double q2 = q[4 * (size_t)p + 2];
    double y[18];
    load_yplane(Y, (size_t)v.NE, (size_t)i, y);
#pragma unroll
    for (int a = 0; a < 6; ++a) acc[21 + a] -= y[3 * a] * qa.x + y[3 * a + 1] * qa.y + y[3 * a + 2] * q2;
    const int len = run[i];
    if (len == 0) continue;
    for (int j = 1; j < len; ++j) {  // rare (rig): fold the run into Z
      double w[18];
      load_yplane(Y, (size_t)v.NE, (size_t)(i + j), w);
#pragma unroll
      for (int k = 0; k < 18; ++k) y[k] += w[k];
    }
    int k = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int bb = a; bb < 6; ++bb)
        acc[k++] += y[3 * a] * y[3 * bb] + y[3 * a + 1] * y[3 * bb + 1] + y[3 * a + 2] * y[3 * bb + 2];
  }
  // fixed-order block reduction
  __shared__ double sh[kRedBlock / 64][27];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 27; ++i) {
    const double t = wave_sum_lane63(acc[i]);
    if (lane == 63) sh[w][i] = t;
  }
  __syncthreads();
  if (threadIdx.x < 27) {
    double t = sh[0][threadIdx.x];
#pragma unroll
    for (int q2 = 1; q2 < kRedBlock / 64; ++q2) t += sh[q2][threadIdx.x];
    partial[27 * (size_t)c + threadIdx.x] = t;
  }
}

// thread per camera: A_c = s U_cc s + D^2 (full 36, kept for the operator), M_c^-1 from
// A_c - sum Y Y^T (6x6 Cholesky + inverse), b_c = s g_c - sum Y q, x = 0, r = b.
__global__ __launch_bounds__(256) void k_pcg_setup(int NC, const double* __restrict__ ug,
                                                   const double* __restrict__ scc, StepScalars sc,
                                                   const double* __restrict__ red /*[NC][27]*/,
                                                   double* __restrict__ Ad, double* __restrict__ Minv,
                                                   double* __restrict__ bvec, double* __restrict__ x,
                                                   double* __restrict__ r, int* __restrict__ fail) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= NC) return;
  const double* u = ug + 27 * (size_t)c;
  const double* rd = red + 27 * (size_t)c;
  double s[6];
#pragma unroll
  for (int a = 0; a < 6; ++a) s[a] = scc[6 * c + a];
  double A[6][6], M[6][6];
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      const int lo = a < b ? a : b, hi = a < b ? b : a;
      double val = s[a] * u[up6(lo, hi)] * s[b];
      if (a == b) {
        const double d = fmin(fmax(val, sc.min_diag), sc.max_diag);
        const double D = sqrt(d / sc.radius);
        val += D * D;
      }
      A[a][b] = val;
      M[a][b] = val - rd[up6(lo, hi)];
    }
  double* ad = Ad + 36 * (size_t)c;
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b) ad[6 * a + b] = A[a][b];
  // Cholesky M = L L^T (lower, in place)
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double d = M[j][j];
#pragma unroll
    for (int k = 0; k < j; ++k) d -= M[j][k] * M[j][k];
    ok = ok && d > 0.0;
    const double l = sqrt(d);
    M[j][j] = l;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      double t = M[i][j];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= M[i][k] * M[j][k];
      M[i][j] = t / l;
    }
  }
  // Li = L^-1 (lower), then M^-1 = Li^T Li
  double Li[6][6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
#pragma unroll
    for (int i = 0; i < 6; ++i) Li[i][j] = 0.0;
    Li[j][j] = 1.0 / M[j][j];
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      double t = 0.0;
#pragma unroll
      for (int k = j; k < i; ++k) t -= M[i][k] * Li[k][j];
      Li[i][j] = t / M[i][i];
    }
  }
  double* mi = Minv + 36 * (size_t)c;
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int b = 0; b < 6; ++b) {
      double t = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k) t += Li[k][a] * Li[k][b];
      ok = ok && isfinite(t);
      mi[6 * a + b] = t;
    }
  if (!ok) atomicOr(fail, 1);
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    const double bv = s[a] * u[21 + a] + rd[21 + a];
    bvec[6 * c + a] = bv;
    r[6 * c + a] = bv;
    x[6 * c + a] = 0.0;
  }
}

// One work-group: z = M^-1 r, rho = r.z, p = z + (rho / rho_prev) p for iteration `iter`
// (p = z when iter == 1). Every thread must call it (block-wide reductions).
__device__ void pcg_direction(int NC, const double* __restrict__ Minv, const double* __restrict__ r,
                              double* __restrict__ z, double* __restrict__ p, PcgState* st, int iter, double* sh) {
  double acc = 0.0;
  for (int c = threadIdx.x; c < NC; c += blockDim.x) {
    const double* mi = Minv + 36 * (size_t)c;
    double rc[6];
#pragma unroll
    for (int a = 0; a < 6; ++a) rc[a] = r[6 * c + a];
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      double t = 0.0;
#pragma unroll
      for (int b = 0; b < 6; ++b) t += mi[6 * a + b] * rc[b];
      z[6 * c + a] = t;
      acc += rc[a] * t;
    }
  }
  const double rho = wg_sum(acc, sh);
  const double rho_prev = st->rho;
  const double beta = iter == 1 ? 0.0 : rho / rho_prev;
  const bool bad = zero_or_inf(rho) || (iter > 1 && zero_or_inf(beta));
  if (!bad) {
    for (int c = threadIdx.x; c < NC; c += blockDim.x) {
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        const int i = 6 * c + a;
        p[i] = iter == 1 ? z[i] : z[i] + beta * p[i];
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    st->iter = iter;
    st->rho = rho;
    if (bad) st->status = kPcgFailure;
  }
}

// one work-group: norm_b, status
__global__ __launch_bounds__(kOneWG) void k_pcg_init(int NC, const double* __restrict__ bvec,
                                                     const int* __restrict__ fail, PcgState* st,
                                                     double eta, int min_iter, int max_iter,
                                                     const double* __restrict__ Minv, const double* __restrict__ r,
                                                     double* __restrict__ z, double* __restrict__ p) {
  __shared__ double sh[kOneWG / 64];
  __shared__ int s_status;
  const int n = 6 * NC;
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += bvec[i] * bvec[i];
  const double nb2 = wg_sum(acc, sh);
  if (threadIdx.x == 0) {
    st->rho = 0.0;
    st->Q0 = 0.0;
    st->alpha = 0.0;
    st->eta = eta;
    st->norm_b = sqrt(nb2);
    st->iter = 0;
    st->min_iter = min_iter;
    st->max_iter = max_iter;
    st->status = fail[0] != 0 ? kPcgFailure : (nb2 == 0.0 ? kPcgSuccess : kPcgRunning);
    if (st->status == kPcgRunning && max_iter <= 0) st->status = kPcgNoConvergence;
    s_status = st->status;
  }
  __syncthreads();
  if (s_status == kPcgRunning) pcg_direction(NC, Minv, r, z, p, st, 1, sh);  // iteration 1
}

// ---- per iteration -------------------------------------------------------------------

// one work-group: z = M^-1 r, rho = r.z, p = z + beta p
// point pass: t_p = sum_e Y_e^T v_cam(e) -> t[NP][4]; lane = point over its SELL slots
// (coalesced planar records of both extrinsic slots)
template <class YT>
__global__ __launch_bounds__(256) void k_pcg_point_pass(DevView v, const YT* __restrict__ Ypm,
                                                        const double* __restrict__ vec,
                                                        double* __restrict__ t, const PcgState* st) {
  if (st->status != kPcgRunning) return;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= v.NP) return;
  const size_t NS = (size_t)v.N;
  const int sl = p >> 6, lane = p & 63;
  const int off = v.slice_off[sl], len = (v.slice_off[sl + 1] - off) >> 6;
  double t0 = 0.0, t1 = 0.0, t2 = 0.0;
  for (int k = 0; k < len; ++k) {
    const int s = off + 64 * k + lane;
    const int4 id = v.obs_idx[s];
    if (id.x < 0) continue;
#pragma unroll
    for (int slot = 0; slot < 2; ++slot) {
      const int e = slot ? id.z : id.y;
      const int c = e >= 0 ? v.ext_col[e] : -1;
      if (c < 0) continue;
      double y[18];
      load_yplane(Ypm + slot * 18 * NS, NS, (size_t)s, y);
      const double2* v2 = reinterpret_cast<const double2*>(vec + 6 * (size_t)c);
      double vc[6];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const double2 w = v2[q];
        vc[2 * q] = w.x;
        vc[2 * q + 1] = w.y;
      }
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        t0 += y[3 * a] * vc[a];
        t1 += y[3 * a + 1] * vc[a];
        t2 += y[3 * a + 2] * vc[a];
      }
    }
  }
  reinterpret_cast<double2*>(t)[2 * (size_t)p] = make_double2(t0, t1);
  reinterpret_cast<double2*>(t)[2 * (size_t)p + 1] = make_double2(t2, 0.0);
}

// Fused matvec for small camera systems (NC <= kFuseCams, e.g. the rig's 79 cameras): one
// pass over the point-major Y records computes t_p = sum_e Y_e^T v_c(e) and then, re-reading
// the point's records (L2-resident by then), adds -Y_e t_p into per-wave camera
// accumulators in LDS. The camera-major copy of Y is not read, so the records cross HBM once
// per product instead of twice (the re-read of a point's records mostly misses L2: 443 us
// per product at C5 fp32 against 240 us for the first half alone and 706 us for the two
// camera/point passes). Each wave owns its accumulator (LDS atomics only between
// the lanes of one instruction, which the LDS resolves in a fixed order), the waves and
// then the work-groups are summed in a fixed order: bitwise reproducible.
constexpr int kFuseCams = 160;
constexpr int kFuseBlock = 256;
template <class YT>
__global__ __launch_bounds__(kFuseBlock) void k_pcg_fused(DevView v, const YT* __restrict__ Ypm,
                                                          const double* __restrict__ vec,
                                                          double* __restrict__ partial, const PcgState* st) {
  extern __shared__ double accs[];  // [kFuseBlock / 64][6 NC]
  if (st->status != kPcgRunning) return;
  const int NC6 = 6 * v.NC, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < (kFuseBlock / 64) * NC6; i += blockDim.x) accs[i] = 0.0;
  __syncthreads();
  double* acc = accs + w * NC6;
  const size_t NS = (size_t)v.N;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < v.NP; p += gridDim.x * blockDim.x) {
    const int sl = p >> 6, lane = p & 63;
    const int off = v.slice_off[sl], len = (v.slice_off[sl + 1] - off) >> 6;
    double t0 = 0.0, t1 = 0.0, t2 = 0.0;
    for (int k = 0; k < len; ++k) {
      const int s = off + 64 * k + lane;
      const int4 id = v.obs_idx[s];
      if (id.x < 0) continue;
#pragma unroll
      for (int slot = 0; slot < 2; ++slot) {
        const int e = slot ? id.z : id.y;
        const int c = e >= 0 ? v.ext_col[e] : -1;
        if (c < 0) continue;
        double y[18];
        load_yplane(Ypm + slot * 18 * NS, NS, (size_t)s, y);
        const double2* v2 = reinterpret_cast<const double2*>(vec + 6 * (size_t)c);
        double vc[6];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const double2 u = v2[q];
          vc[2 * q] = u.x;
          vc[2 * q + 1] = u.y;
        }
#pragma unroll
        for (int a = 0; a < 6; ++a) {
          t0 += y[3 * a] * vc[a];
          t1 += y[3 * a + 1] * vc[a];
          t2 += y[3 * a + 2] * vc[a];
        }
      }
    }
    for (int k = 0; k < len; ++k) {
      const int s = off + 64 * k + lane;
      const int4 id = v.obs_idx[s];
      if (id.x < 0) continue;
#pragma unroll
      for (int slot = 0; slot < 2; ++slot) {
        const int e = slot ? id.z : id.y;
        const int c = e >= 0 ? v.ext_col[e] : -1;
        if (c < 0) continue;
        double y[18];
        load_yplane(Ypm + slot * 18 * NS, NS, (size_t)s, y);
#pragma unroll
        for (int a = 0; a < 6; ++a)
          atomicAdd(acc + 6 * c + a, -(y[3 * a] * t0 + y[3 * a + 1] * t1 + y[3 * a + 2] * t2));
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NC6; i += blockDim.x) {
    double x = accs[i];
#pragma unroll
    for (int q = 1; q < kFuseBlock / 64; ++q) x += accs[q * NC6 + i];
    partial[(size_t)blockIdx.x * NC6 + i] = x;
  }
}

// w[i] = sum over the G work-group partials, fixed order (one block per output)
__global__ __launch_bounds__(256) void k_pcg_fused_final(int G, int NC6, const double* __restrict__ partial,
                                                         double* __restrict__ w, const PcgState* st) {
  if (st->status != kPcgRunning) return;
  const int i = blockIdx.x;
  double x = 0.0;
  for (int b = threadIdx.x; b < G; b += blockDim.x) x += partial[(size_t)b * NC6 + i];
  __shared__ double sh[4];
  const double t = wave_sum_lane63(x);
  if ((threadIdx.x & 63) == 63) sh[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) w[i] = ((sh[0] + sh[1]) + sh[2]) + sh[3];
}

// camera pass: per chunk of positions -sum Y_pos t_pt(pos) -> partial[chunk][6]
template <class YT>
__global__ __launch_bounds__(256) void k_pcg_cam_pass(DevView v, const int* __restrict__ chunk_beg,
                                                      const YT* __restrict__ Y, const double* __restrict__ t,
                                                      double* __restrict__ partial, const PcgState* st) {
  if (st->status != kPcgRunning) return;
  const int c = blockIdx.x;
  const int b = chunk_beg[c], e = chunk_beg[c + 1];
  double acc[6] = {0, 0, 0, 0, 0, 0};
  for (int i = b + threadIdx.x; i < e; i += blockDim.x) {
    const int p = v.cm_pt[i];
    const double2 ta = reinterpret_cast<const double2*>(t)[2 * (size_t)p];
    const double t2 = t[4 * (size_t)p + 2];
    double y[18];
    load_yplane(Y, (size_t)v.NE, (size_t)i, y);
#pragma unroll
    for (int a = 0; a < 6; ++a) acc[a] -= y[3 * a] * ta.x + y[3 * a + 1] * ta.y + y[3 * a + 2] * t2;
  }
  __shared__ double sh[kRedBlock / 64][6];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double x = wave_sum_lane63(acc[i]);
    if (lane == 63) sh[w][i] = x;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    double x = sh[0][threadIdx.x];
#pragma unroll
    for (int q = 1; q < kRedBlock / 64; ++q) x += sh[q][threadIdx.x];
    partial[6 * (size_t)c + threadIdx.x] = x;
  }
}

// (A_cc + cross) vec + w for camera c, component-wise into out[6]
// S_cc v_c + w_c + sum of the cross terms of camera c, by the L consecutive lanes s of a
// group (L = 16 with cross blocks, else 1): lane s takes every L-th cross block of c, the
// diagonal goes to lane 0, and the L partials are combined by a fixed xor tree (every lane
// of the group ends with the same sum). Cameras with ~60 cross blocks (rig arc cameras) no
// longer serialise one lane.
// wc: camera c's 6 values of the Y part (w + 6 c, or a work-group's own sum of the partials)
__device__ __forceinline__ void apply_cam8(int c, int s, int L, const double* __restrict__ Ad,
                                           const double* __restrict__ vec, const double* wc,
                                           const int* __restrict__ xptr, const int* __restrict__ xlist,
                                           const int2* __restrict__ xcam, const double* __restrict__ X,
                                           const double* __restrict__ scc, double (&out)[6]) {
#pragma unroll
  for (int a = 0; a < 6; ++a) out[a] = 0.0;
  if (c >= 0) {
    if (s == 0) {
      const double* ad = Ad + 36 * (size_t)c;
      double vc[6];
#pragma unroll
      for (int b = 0; b < 6; ++b) vc[b] = vec[6 * c + b];
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        double t = wc[a];
#pragma unroll
        for (int b = 0; b < 6; ++b) t += ad[6 * a + b] * vc[b];
        out[a] = t;
      }
    }
    if (xptr) {
      double cr[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
      for (int j = xptr[c] + s; j < xptr[c + 1]; j += L) {
        const int code = xlist[j], k = code >> 1;
        const int2 cc = xcam[k];  // X_k = Jc0^T Jc1, block (c0, c1)
        const double* xk = X + 36 * (size_t)k;
        const bool first = (code & 1) == 0;  // c == c0: (s0 X s1) v_c1, else (s0 X s1)^T v_c0
        const int o = first ? cc.y : cc.x;
        double sv[6];
#pragma unroll
        for (int b = 0; b < 6; ++b) sv[b] = scc[6 * o + b] * vec[6 * o + b];
#pragma unroll
        for (int a = 0; a < 6; ++a) {
          double t = 0.0;
#pragma unroll
          for (int b = 0; b < 6; ++b) t += (first ? xk[6 * a + b] : xk[6 * b + a]) * sv[b];
          cr[a] += t;
        }
      }
#pragma unroll
      for (int a = 0; a < 6; ++a) out[a] += scc[6 * c + a] * cr[a];
    }
  }
  for (int m = 1; m < L; m <<= 1)
#pragma unroll
    for (int a = 0; a < 6; ++a) out[a] += __shfl_xor(out[a], m, L);
}

// one work-group. mode 0: q = S p, alpha, x += alpha p, r -= alpha q, Q-test
//                 mode 1: q = S p, alpha, x += alpha p (r recomputed by mode 2)
//                 mode 2: r = b - S x, Q-test
__global__ __launch_bounds__(kOneWG) void k_pcg_update(int NC, int mode, const double* __restrict__ Ad,
                                                       const double* __restrict__ w,
                                                       const int* __restrict__ xptr, const int* __restrict__ xlist,
                                                       const int2* __restrict__ xcam, const double* __restrict__ X,
                                                       const double* __restrict__ scc, const double* __restrict__ bvec,
                                                       double* __restrict__ p, double* __restrict__ q,
                                                       double* __restrict__ x, double* __restrict__ r,
                                                       PcgState* st, const double* __restrict__ Minv,
                                                       double* __restrict__ z) {
  __shared__ double sh[kOneWG / 64];
  __shared__ int s_status;
  if (st->status != kPcgRunning) return;
  int status = kPcgRunning;
  const int L = xptr ? 16 : 1;  // lanes per camera
  const int s8 = threadIdx.x & (L - 1), cpp = blockDim.x / L;
  const int cam_rounds = (NC + cpp - 1) / cpp;
  if (mode != 2) {
    double acc = 0.0;
    for (int rr = 0; rr < cam_rounds; ++rr) {
      const int c = rr * cpp + threadIdx.x / L;
      double o[6];
      apply_cam8(c < NC ? c : -1, s8, L, Ad, p, c < NC ? w + 6 * c : nullptr, xptr, xlist, xcam, X, scc, o);
      if (c < NC && s8 == 0) {
#pragma unroll
        for (int a = 0; a < 6; ++a) {
          q[6 * c + a] = o[a];
          acc += p[6 * c + a] * o[a];
        }
      }
    }
    const double pq = wg_sum(acc, sh);
    if (pq <= 0.0 || isinf(pq)) {
      // Ceres: "Matrix is indefinite, no more progress can be made" — keep x
      if (threadIdx.x == 0) st->status = kPcgNoConvergence;
      return;
    }
    const double alpha = st->rho / pq;
    if (isinf(alpha)) {
      if (threadIdx.x == 0) st->status = kPcgFailure;
      return;
    }
    for (int c = threadIdx.x; c < NC; c += blockDim.x) {
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        const int i = 6 * c + a;
        x[i] += alpha * p[i];
        if (mode == 0) r[i] -= alpha * q[i];
      }
    }
    if (mode == 1) return;
  } else {
    for (int rr = 0; rr < cam_rounds; ++rr) {
      const int c = rr * cpp + threadIdx.x / L;
      double o[6];
      apply_cam8(c < NC ? c : -1, s8, L, Ad, x, c < NC ? w + 6 * c : nullptr, xptr, xlist, xcam, X, scc, o);
      if (c < NC && s8 == 0) {
#pragma unroll
        for (int a = 0; a < 6; ++a) r[6 * c + a] = bvec[6 * c + a] - o[a];
      }
    }
  }
  double acc = 0.0;
  for (int c = threadIdx.x; c < NC; c += blockDim.x) {
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      const int i = 6 * c + a;
      acc += x[i] * (bvec[i] + r[i]);
    }
  }
  const double Q1 = -wg_sum(acc, sh);
  const int iter = st->iter;
  if (threadIdx.x == 0) {
    const double zeta = iter * (Q1 - st->Q0) / Q1;
    if (zeta < st->eta && iter >= st->min_iter) status = kPcgSuccess;
    else if (iter >= st->max_iter) status = kPcgNoConvergence;
    st->Q0 = Q1;
    st->status = status;
    s_status = status;
  }
  __syncthreads();
  // still running: the next iteration's direction, in the same launch
  if (s_status == kPcgRunning) pcg_direction(NC, Minv, r, z, p, st, iter + 1, sh);
}

// ---- multi-work-group CG update ---------------------------------------------------------
// The single-work-group update above pulls Ad, M^-1 and five vectors through one CU (~50
// us at NC = 999). Here the camera-wise work is spread over 64-thread work-groups and each
// global dot product is finished by the last work-group to arrive (partials stored
// write-through and drained before one atomic count, read back with atomic loads, summed
// in work-group order: deterministic, no fences), so the scalar recurrences stay on the
// device. Two launches per CG iteration:
//   k_cg_q      q = S p (Y part w + diagonal + cross terms), pq -> alpha (mode 0/1);
//               mode 2: r = b - S x
//   k_cg_xr     x += alpha p, r -= alpha q (mode 0), Q-test, z = M^-1 r, rho -> beta, iter;
//               for small camera sets the last work-group then p = z + beta p (z written
//               with agent-scope stores); otherwise a third launch, k_cg_p
constexpr int kCgBlock = 64;

// sum of v over the grid, valid in the last-arriving work-group (returns true there)
template <int K>
__device__ __forceinline__ bool grid_sum_last(double (&v)[K], double* __restrict__ partial, unsigned* __restrict__ cnt,
                                              double (&out)[K]) {
  __shared__ int last;
#pragma unroll
  for (int i = 0; i < K; ++i) v[i] = wave_sum_lane63(v[i]);  // one wave per work-group
  if (threadIdx.x == 63) {
#pragma unroll
    for (int i = 0; i < K; ++i)
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(partial) + K * (size_t)blockIdx.x + i,
                         (unsigned long long)__double_as_longlong(v[i]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return false;
  const unsigned long long* pp = reinterpret_cast<const unsigned long long*>(partial);
#pragma unroll
  for (int i = 0; i < K; ++i) {
    double s = 0.0;
    for (int b = threadIdx.x; b < (int)gridDim.x; b += blockDim.x)
      s += __longlong_as_double((long long)__hip_atomic_load(pp + K * (size_t)b + i, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT));
    out[i] = wave_sum_lane63(s);  // lane 63 holds the total
  }
  if (threadIdx.x == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

__global__ __launch_bounds__(kCgBlock) void k_cg_q(int NC, int mode, int L, const double* __restrict__ Ad,
                                                   const double* __restrict__ w, const int* __restrict__ xptr,
                                                   const int* __restrict__ xlist, const int2* __restrict__ xcam,
                                                   const double* __restrict__ X, const double* __restrict__ scc,
                                                   const double* __restrict__ bvec, const double* __restrict__ p,
                                                   double* __restrict__ q, const double* __restrict__ x,
                                                   double* __restrict__ r, PcgState* st, double* __restrict__ partial,
                                                   unsigned* __restrict__ cnt, const double* __restrict__ wpart,
                                                   int G) {
  if (st->status != kPcgRunning) return;
  const int s8 = threadIdx.x & (L - 1);
  const int c0 = blockIdx.x * (kCgBlock / L) + threadIdx.x / L;
  const int c = c0 < NC ? c0 : -1;
  // wpart (L = 64, one camera per work-group): the product's G work-group partials summed
  // here in a fixed order instead of by a launch of their own
  __shared__ double wsh[6];
  if (wpart) {
    double a6[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    if (c >= 0)
      for (int g = threadIdx.x; g < G; g += kCgBlock)
#pragma unroll
        for (int a = 0; a < 6; ++a) a6[a] += wpart[(size_t)g * 6 * NC + 6 * c + a];
    wave_sums_transposed<6>(a6, wsh);
    __syncthreads();
  }
  double o[6];
  apply_cam8(c, s8, L, Ad, mode == 2 ? x : p, wpart ? wsh : (c >= 0 ? w + 6 * c : nullptr), xptr, xlist, xcam, X,
             scc, o);
  double acc[1] = {0.0};
  if (c >= 0 && s8 == 0) {
    if (mode == 2) {
#pragma unroll
      for (int a = 0; a < 6; ++a) r[6 * c + a] = bvec[6 * c + a] - o[a];
    } else {
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        q[6 * c + a] = o[a];
        acc[0] += p[6 * c + a] * o[a];
      }
    }
  }
  if (mode == 2) return;
  double pq[1];
  if (!grid_sum_last<1>(acc, partial, cnt, pq)) return;
  if (threadIdx.x == 63) {
    if (pq[0] <= 0.0 || isinf(pq[0])) {
      st->status = kPcgNoConvergence;  // Ceres: matrix indefinite, keep x
    } else {
      const double alpha = st->rho / pq[0];
      if (isinf(alpha)) st->status = kPcgFailure;
      st->alpha = alpha;
    }
  }
}

// mode 0: x, r update + Q-test + direction scalars; 1: x update only; 2: Q-test + direction
__global__ __launch_bounds__(kCgBlock) void k_cg_xr(int NC, int mode, const double* __restrict__ bvec,
                                                    double* __restrict__ p, const double* __restrict__ q,
                                                    double* __restrict__ x, double* __restrict__ r,
                                                    const double* __restrict__ Minv, double* __restrict__ z,
                                                    PcgState* st, double* __restrict__ partial,
                                                    unsigned* __restrict__ cnt, int fold_p) {
  if (st->status != kPcgRunning) return;
  const int c = blockIdx.x * kCgBlock + threadIdx.x;
  double acc[2] = {0.0, 0.0};  // x.(b + r), r.z
  if (c < NC) {
    double xc[6], rc[6];
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      xc[a] = x[6 * c + a];
      rc[a] = r[6 * c + a];
    }
    if (mode != 2) {
      const double alpha = st->alpha;
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        xc[a] += alpha * p[6 * c + a];
        x[6 * c + a] = xc[a];
        if (mode == 0) {
          rc[a] -= alpha * q[6 * c + a];
          r[6 * c + a] = rc[a];
        }
      }
    }
    if (mode != 1) {
#pragma unroll
      for (int a = 0; a < 6; ++a) acc[0] += xc[a] * (bvec[6 * c + a] + rc[a]);
      const double* mi = Minv + 36 * (size_t)c;
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        double t = 0.0;
#pragma unroll
        for (int b = 0; b < 6; ++b) t += mi[6 * a + b] * rc[b];
        // agent scope: the last-arriving work-group reads every z for p = z + beta p
        __hip_atomic_store(z + 6 * c + a, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        acc[1] += rc[a] * t;
      }
    }
  }
  if (mode == 1) return;
  double sums[2];
  if (!grid_sum_last<2>(acc, partial, cnt, sums)) return;
  __shared__ double beta_s;
  __shared__ int run_s;
  if (threadIdx.x == 63) {
    run_s = 0;
    const double Q1 = -sums[0];
    const int iter = st->iter;
    int status = kPcgRunning;
    const double zeta = iter * (Q1 - st->Q0) / Q1;
    if (zeta < st->eta && iter >= st->min_iter) status = kPcgSuccess;
    else if (iter >= st->max_iter) status = kPcgNoConvergence;
    st->Q0 = Q1;
    if (status == kPcgRunning) {  // the next iteration's direction scalars
      const double rho = sums[1];
      const double beta = rho / st->rho;
      if (zero_or_inf(rho) || zero_or_inf(beta)) status = kPcgFailure;
      st->pad[0] = beta;
      st->rho = rho;
      st->iter = iter + 1;
      beta_s = beta;
    }
    st->status = status;
    run_s = status == kPcgRunning;
  }
  __syncthreads();
  // p = z + beta p by the last work-group, every z of this launch now written (small
  // camera sets; otherwise k_cg_p spreads it)
  if (fold_p && run_s)
    for (int i = threadIdx.x; i < 6 * NC; i += blockDim.x)
      p[i] = __hip_atomic_load(z + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + beta_s * p[i];
}


__global__ __launch_bounds__(256) void k_cg_p(int n, const double* __restrict__ z, double* __restrict__ p,
                                              const PcgState* st) {
  if (st->status != kPcgRunning) return;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = z[i] + st->pad[0] * p[i];
}

// ---- launchers -------------------------------------------------------------------------

void launch_pcg_diag_rhs_partial(hipStream_t s, const DevView& v, int nchunk, const int* chunk_beg,
                                 const int* run, YBufs Y, const double* q, double* partial) {
  if (nchunk <= 0) return;
  if (Y.f32)
    k_pcg_diag_rhs_partial<float><<<nchunk, kRedBlock, 0, s>>>(v, chunk_beg, run, (const float*)Y.cm, q, partial);
  else
    k_pcg_diag_rhs_partial<double><<<nchunk, kRedBlock, 0, s>>>(v, chunk_beg, run, (const double*)Y.cm, q,
                                                                partial);
}

void launch_pcg_setup(hipStream_t s, int NC, const double* ug, const double* scale_c, StepScalars sc,
                      const double* red, double* Ad, double* Minv, double* bvec, double* x, double* r,
                      int* fail) {
  if (NC <= 0) return;
  k_pcg_setup<<<grid_for(NC, 256, 1 << 20), 256, 0, s>>>(NC, ug, scale_c, sc, red, Ad, Minv, bvec, x, r, fail);
}

void launch_pcg_init(hipStream_t s, int NC, const double* bvec, const int* fail, PcgState* st, double eta,
                     int min_iter, int max_iter, const double* Minv, const double* r, double* z, double* p) {
  k_pcg_init<<<1, kOneWG, 0, s>>>(NC, bvec, fail, st, eta, min_iter, max_iter, Minv, r, z, p);
}


bool pcg_fused_fits(int NC) { return NC > 0 && NC <= kFuseCams; }
int pcg_fused_grid(int NP, int ncu) { return std::max(1, std::min((NP + kFuseBlock - 1) / kFuseBlock, 4 * ncu)); }

void launch_pcg_fused(hipStream_t s, const DevView& v, YBufs Y, const double* vec, double* partial, double* w,
                      int grid, const PcgState* st) {
  const int NC6 = 6 * v.NC;
  const size_t lds = sizeof(double) * (kFuseBlock / 64) * NC6;
  if (Y.f32) k_pcg_fused<float><<<grid, kFuseBlock, lds, s>>>(v, (const float*)Y.pm, vec, partial, st);
  else k_pcg_fused<double><<<grid, kFuseBlock, lds, s>>>(v, (const double*)Y.pm, vec, partial, st);
  k_pcg_fused_final<<<NC6, 256, 0, s>>>(grid, NC6, partial, w, st);
}

void launch_pcg_fused_final(hipStream_t s, int grid, int NC6, const double* partial, double* w, const PcgState* st) {
  k_pcg_fused_final<<<NC6, 256, 0, s>>>(grid, NC6, partial, w, st);
}

void launch_pcg_matvec_passes(hipStream_t s, const DevView& v, int nchunk, const int* chunk_beg, YBufs Y,
                              const double* vec, double* t, double* partial, const PcgState* st) {
  const int g = grid_for(v.NP, 256, 1 << 20);
  if (Y.f32) {
    if (v.NP > 0) k_pcg_point_pass<float><<<g, 256, 0, s>>>(v, (const float*)Y.pm, vec, t, st);
    if (nchunk > 0)
      k_pcg_cam_pass<float><<<nchunk, kRedBlock, 0, s>>>(v, chunk_beg, (const float*)Y.cm, t, partial, st);
  } else {
    if (v.NP > 0) k_pcg_point_pass<double><<<g, 256, 0, s>>>(v, (const double*)Y.pm, vec, t, st);
    if (nchunk > 0)
      k_pcg_cam_pass<double><<<nchunk, kRedBlock, 0, s>>>(v, chunk_beg, (const double*)Y.cm, t, partial, st);
  }
}

void launch_cg_update(hipStream_t s, int NC, int mode, const double* Ad, const double* w, const int* xptr,
                      const int* xlist, const int2* xcam, const double* X, const double* scale_c,
                      const double* bvec, double* p, double* q, double* x, double* r, PcgState* st,
                      const double* Minv, double* z, double* partial, unsigned* cnt, const double* wpart,
                      int wpart_g) {
  if (NC <= 0) return;
  // with cross blocks a wave per camera: its cross blocks' loads all in flight at once (the
  // rig: 63 per arc camera; 16 lanes per camera walked them in 4 dependent rounds)
  const int L = xptr ? 64 : 1;
  const int gq = (NC + kCgBlock / L - 1) / (kCgBlock / L), gx = (NC + kCgBlock - 1) / kCgBlock;
  if (mode != 2)
    k_cg_q<<<gq, kCgBlock, 0, s>>>(NC, mode, L, Ad, w, xptr, xlist, xcam, X, scale_c, bvec, p, q, x, r, st, partial, cnt,
                                   L == 64 ? wpart : nullptr, wpart_g);
  else
    k_cg_q<<<gq, kCgBlock, 0, s>>>(NC, 2, L, Ad, w, xptr, xlist, xcam, X, scale_c, bvec, p, q, x, r, st, partial, cnt,
                                   L == 64 ? wpart : nullptr, wpart_g);
  const int fold_p = 6 * NC <= 2048;  // one work-group does p = z + beta p in <= 32 passes
  k_cg_xr<<<gx, kCgBlock, 0, s>>>(NC, mode, bvec, p, q, x, r, Minv, z, st, partial, cnt, fold_p);
  if (mode != 1 && !fold_p) k_cg_p<<<(6 * NC + 255) / 256, 256, 0, s>>>(6 * NC, z, p, st);
}
// the CG update's grid partials: k_cg_q writes K = 1 per work-group over NC / (kCgBlock / L)
// work-groups (L = 64 with cross blocks: one camera per work-group, NC partials), then
// k_cg_xr K = 2 per work-group over ceil(NC / kCgBlock). (Sized for the earlier L = 16,
// 2 ceil(NC / 4), this ran past its end by NC / 2 doubles on the rig, which the allocator's
// padding hid until buffers were packed.)
int cg_partial_size(int NC) { return NC + 2 * ((NC + kCgBlock - 1) / kCgBlock); }

void launch_pcg_update(hipStream_t s, int NC, int mode, const double* Ad, const double* w, const int* xptr,
                       const int* xlist, const int2* xcam, const double* X, const double* scale_c,
                       const double* bvec, double* p, double* q, double* x, double* r, PcgState* st,
                       const double* Minv, double* z) {
  k_pcg_update<<<1, kOneWG, 0, s>>>(NC, mode, Ad, w, xptr, xlist, xcam, X, scale_c, bvec, p, q, x, r, st, Minv, z);
}

// Loads this translation unit's code object on the current device now: otherwise the first
// launch of any of its kernels pays for it (10-40 ms, inside a process's first LM iteration).
void warm_pcg() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(k_pcg_setup));
}

}  // namespace dab
