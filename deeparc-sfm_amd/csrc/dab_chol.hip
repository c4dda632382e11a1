// dab_chol.hip — dense Cholesky of the reduced camera system (SURVEY §8a row a7:
// DENSE_SCHUR's "dense Cholesky of S", sfm.cc:67) plus the triangular solves.
//
// S is stored row-major, lower triangle, with the right-hand side appended as row n
// (the augmented matrix [[S, b], [b^T, *]]). Factoring the first n pivots of the
// augmented matrix leaves L in rows 0..n-1 and z = L^-1 b in row n, so the forward
// substitution rides along with the factorisation. Blocked right-looking, NB = 64:
//   k_potrf_inv  factor + invert the 64x64 diagonal block (one workgroup, LDS-resident,
//                one barrier per pivot; inverse by 4 lanes per column, no barriers)
//   k_trsm_inv   panel rows <- rows L_kk^-T (product with the stored inverse; every row
//                independent, 16 rows per workgroup to fill the chip)
//   k_syrk_mfma  trailing update C -= P P^T on lower 64x64 tiles with fp64 MFMA
//                (v_mfma_f64_16x16x4_f64, 4 waves x 32x32 quadrants, P tiles in LDS)
// Back substitution L^T y = z: one launch per block, y_k = L_kk^-T z_k from the stored
// inverse followed by the block-column update of z[0:k].
#include <hip/hip_runtime.h>

#include "dab_kernels.h"

namespace dab {

constexpr int NB = 64;
constexpr int kThreads = 256;
constexpr int LDP = 66;  // padded LDS row stride (doubles): conflict-free fragment reads

typedef double dbl4 __attribute__((ext_vector_type(4)));

struct CholCtx {
  double* linv = nullptr;  // [nblk][NB][NB] inverses of the diagonal blocks
  size_t linv_blocks = 0;
  // the ~5 x n/64 dependent launches are captured once per (n, buffers) and replayed
  hipGraphExec_t exec = nullptr;
  int g_n = -1, g_lda = -1;
  const void *g_A = nullptr, *g_y = nullptr, *g_flag = nullptr;
};

CholCtx* chol_create() { return new CholCtx(); }
void chol_destroy(CholCtx* c) {
  if (!c) return;
  if (c->exec) (void)hipGraphExecDestroy(c->exec);
  if (c->linv) (void)hipFree(c->linv);
  delete c;
}

__device__ __forceinline__ double bcast(double v, int lane) {  // lane: compile-time constant
  const int2 p = *reinterpret_cast<int2*>(&v);
  int2 r;
  r.x = __builtin_amdgcn_readlane(p.x, lane);
  r.y = __builtin_amdgcn_readlane(p.y, lane);
  return *reinterpret_cast<double*>(&r);
}

// Factor A[k:k+kb, k:k+kb] (lower) in place (identity padding beyond kb). One wave, lane =
// row held in registers, fully unrolled. VAR 0: the pivot column is broadcast with
// v_readlane; VAR 1: through LDS (one ds_write per lane, then ds_read_b128 broadcasts).
template <int VAR>
__global__ __launch_bounds__(64) void k_potrf(double* __restrict__ A, int lda, int k, int kb,
                                              int* __restrict__ flag) {
  __shared__ double col[NB];
  const int m = threadIdx.x;
  double a[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    double v = (m == j) ? 1.0 : 0.0;
    if (m < kb && j < kb && j <= m) v = A[(size_t)(k + m) * lda + k + j];
    a[j] = v;
  }
  bool bad = false;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    double d;
    if constexpr (VAR == 0) {
      d = bcast(a[j], j);  // pivot a_jj (updated)
    } else {
      if (m == j) col[0] = a[j];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      d = col[0];
      __builtin_amdgcn_wave_barrier();
    }
    bad |= !(d > 0.0) || !isfinite(d);
    const double sd = sqrt(d);
    const double lmj = (m == j) ? sd : a[j] / sd;  // L[m][j] (meaningful for m >= j)
    a[j] = lmj;
    if constexpr (VAR == 0) {
#pragma unroll
      for (int l = j + 1; l < NB; ++l) {
        const double llj = bcast(lmj, l);
        if (m >= l) a[l] -= lmj * llj;
      }
    } else {
      col[m] = lmj;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int l = j + 1; l < NB; ++l) {
        const double llj = col[l];
        if (m >= l) a[l] -= lmj * llj;
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (m == 0 && bad) atomicOr(flag, 1);
  if (m < kb) {
#pragma unroll
    for (int j = 0; j < NB; ++j)
      if (j <= m && j < kb) A[(size_t)(k + m) * lda + k + j] = a[j];
  }
}

// Inverse of the factored diagonal block L_kk (lower, identity-padded beyond kb) by
// recursive doubling: the eight 8x8 diagonal blocks by substitution (one lane per
// column), then three levels X21 = -X22 (L21 X11) of small parallel products. The
// dependent chain is 8 substitution steps + 6 barriers instead of 64 pivot steps.
__global__ __launch_bounds__(kThreads) void k_trinv(const double* __restrict__ A, int lda, int k, int kb,
                                                    double* __restrict__ linv) {
  __shared__ double L[NB][NB + 1];
  __shared__ double X[NB][NB + 1];
  __shared__ double T[NB][NB + 1];
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < NB * NB / kThreads; ++q) {
    const int idx = tid + q * kThreads, i = idx >> 6, j = idx & 63;
    double v = (i == j) ? 1.0 : 0.0;
    if (i < kb && j <= i) v = A[(size_t)(k + i) * lda + k + j];
    L[i][j] = v;
    X[i][j] = 0.0;
  }
  __syncthreads();
  if (tid < NB) {  // level 0: block b = tid / 8, column c = tid % 8
    const int b = tid >> 3, c = tid & 7, o = 8 * b;
    double x[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      double s = (r == c) ? 1.0 : 0.0;
#pragma unroll
      for (int mm = 0; mm < r; ++mm) s -= L[o + r][o + mm] * x[mm];
      x[r] = (r >= c) ? s / L[o + r][o + r] : 0.0;
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) X[o + r][o + c] = x[r];
  }
  __syncthreads();
#pragma unroll
  for (int h = 8; h < NB; h *= 2) {
    // pairs of h-blocks at offsets o = 2h q: T = L21 X11, then X21 = -X22 T
    const int nout = NB / (2 * h) * h * h;  // outputs per phase over all pairs
    for (int e = tid; e < nout; e += kThreads) {
      const int pq = e / (h * h), rem = e - pq * h * h, i = rem / h, j = rem - (rem / h) * h;
      const int o = 2 * h * pq;
      double s = 0.0;
      for (int mm = j; mm < h; ++mm) s += L[o + h + i][o + mm] * X[o + mm][o + j];
      T[o + h + i][o + j] = s;
    }
    __syncthreads();
    for (int e = tid; e < nout; e += kThreads) {
      const int pq = e / (h * h), rem = e - pq * h * h, i = rem / h, j = rem - (rem / h) * h;
      const int o = 2 * h * pq;
      double s = 0.0;
      for (int mm = 0; mm <= i; ++mm) s += X[o + h + i][o + h + mm] * T[o + h + mm][o + j];
      X[o + h + i][o + j] = -s;
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < NB * NB / kThreads; ++q) {
    const int idx = tid + q * kThreads;
    linv[idx] = X[idx >> 6][idx & 63];
  }
}

// rows [r0, r1): A[i, k:k+kb] <- A[i, k:k+kb] Linv^T ; 16 rows per workgroup
constexpr int TR = 16;
__global__ __launch_bounds__(kThreads) void k_trsm_inv(double* __restrict__ A, int lda, int k, int kb, int r0,
                                                       int r1, const double* __restrict__ linv) {
  __shared__ double P[TR][NB + 1];
  __shared__ double Li[NB][NB + 1];
  const int tid = threadIdx.x;
  const int row0 = r0 + blockIdx.x * TR;
#pragma unroll
  for (int q = 0; q < NB * NB / kThreads; ++q) {
    const int idx = tid + q * kThreads;
    Li[idx >> 6][idx & 63] = linv[idx];
  }
#pragma unroll
  for (int q = 0; q < TR * NB / kThreads; ++q) {
    const int idx = tid + q * kThreads, i = idx >> 6, j = idx & 63;
    P[i][j] = (row0 + i < r1 && j < kb) ? A[(size_t)(row0 + i) * lda + k + j] : 0.0;
  }
  __syncthreads();
  const int rr = tid >> 4;  // 16 rows x 16 threads, 4 outputs each
  double out[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = (tid & 15) + 16 * q;
    double s = 0.0;
    for (int mm = 0; mm <= j; ++mm) s += P[rr][mm] * Li[j][mm];
    out[q] = s;
  }
  if (row0 + rr < r1) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = (tid & 15) + 16 * q;
      if (j < kb) A[(size_t)(row0 + rr) * lda + k + j] = out[q];
    }
  }
}

// trailing update on lower 64x64 tiles of the m x m matrix at (r0, r0):
//   C[i][j] -= sum_kk P[i][kk] P[j][kk], P = A[r0.., k..k+kb)
__global__ __launch_bounds__(kThreads) void k_syrk_mfma(double* __restrict__ A, int lda, int r0, int m, int k,
                                                        int kb) {
  __shared__ double Pa[NB * LDP];
  __shared__ double Pb[NB * LDP];
  const int t = blockIdx.x;
  int bi = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((bi + 1) * (bi + 2) / 2 <= t) ++bi;
  while (bi * (bi + 1) / 2 > t) --bi;
  const int bj = t - bi * (bi + 1) / 2;
  const int tid = threadIdx.x;
  const bool diag = bi == bj;
  const int w = tid >> 6, lane = tid & 63;
  const int wr = w >> 1, wc = w & 1;  // 32x32 quadrant of the tile
  const bool skip = diag && wr < wc;  // strictly upper quadrant of a diagonal tile
  const int li = lane & 15, lk = lane >> 4;
  // the accumulators start as the C tile (issued first, so its HBM latency overlaps the
  // panel staging); the MFMAs then add -P_i P_j^T
  dbl4 acc[2][2];
#pragma unroll
  for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
    for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int row = bi * NB + wr * 32 + a2 * 16 + lk + 4 * reg;
        const int col = bj * NB + wc * 32 + b2 * 16 + li;
        acc[a2][b2][reg] = (!skip && row < m && col < m) ? A[(size_t)(r0 + row) * lda + r0 + col] : 0.0;
      }
  // coalesced tile loads: 8 rows per pass, 32 double2 per row
#pragma unroll
  for (int q = 0; q < NB / 8; ++q) {
    const int rr = (tid >> 5) + 8 * q, c2 = tid & 31;
    const int ra = bi * NB + rr, rb = bj * NB + rr;
    double2 va = make_double2(0.0, 0.0), vb = make_double2(0.0, 0.0);
    if (ra < m) {
      const double* src = A + (size_t)(r0 + ra) * lda + k + 2 * c2;
      va.x = 2 * c2 < kb ? src[0] : 0.0;
      va.y = 2 * c2 + 1 < kb ? src[1] : 0.0;
    }
    if (!diag && rb < m) {
      const double* src = A + (size_t)(r0 + rb) * lda + k + 2 * c2;
      vb.x = 2 * c2 < kb ? src[0] : 0.0;
      vb.y = 2 * c2 + 1 < kb ? src[1] : 0.0;
    }
    *reinterpret_cast<double2*>(&Pa[rr * LDP + 2 * c2]) = va;
    if (!diag) *reinterpret_cast<double2*>(&Pb[rr * LDP + 2 * c2]) = vb;
  }
  __syncthreads();
  const double* PB = diag ? Pa : Pb;
  if (skip) return;
#pragma unroll 4
  for (int ks = 0; ks < NB / 4; ++ks) {
    double fa[2], fb[2];
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2) fa[a2] = -Pa[(wr * 32 + a2 * 16 + li) * LDP + ks * 4 + lk];
#pragma unroll
    for (int b2 = 0; b2 < 2; ++b2) fb[b2] = PB[(wc * 32 + b2 * 16 + li) * LDP + ks * 4 + lk];
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
      for (int b2 = 0; b2 < 2; ++b2)
        acc[a2][b2] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[a2], fb[b2], acc[a2][b2], 0, 0, 0);
  }
  // D layout (f64 16x16x4): col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
  for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
    for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int row = bi * NB + wr * 32 + a2 * 16 + lk + 4 * reg;
        const int col = bj * NB + wc * 32 + b2 * 16 + li;
        if (row < m && col < m) A[(size_t)(r0 + row) * lda + r0 + col] = acc[a2][b2][reg];
      }
}

// back substitution step for block [k, k+kb): y_k = Linv^T z_k (a 64x64 matvec with the
// stored inverse), then z[0:k] -= L[k:k+kb, 0:k]^T y_k
__global__ __launch_bounds__(kThreads) void k_trsv_back(const double* __restrict__ A, int lda, int k, int kb,
                                                        const double* __restrict__ linv,
                                                        double* __restrict__ z, double* __restrict__ y) {
  __shared__ double Li[NB][NB + 1];
  __shared__ double zz[NB];
  __shared__ double yy[NB];
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < NB * NB / kThreads; ++q) {
    const int idx = tid + q * kThreads;
    Li[idx >> 6][idx & 63] = linv[idx];
  }
  if (tid < NB) zz[tid] = tid < kb ? z[k + tid] : 0.0;
  __syncthreads();
  if (tid < NB) {
    double s = 0.0;
#pragma unroll 8
    for (int mm = 0; mm < NB; ++mm) s += (mm >= tid ? Li[mm][tid] : 0.0) * zz[mm];
    yy[tid] = s;
  }
  __syncthreads();
  if (blockIdx.x == 0 && tid < kb) y[k + tid] = yy[tid];
  // 64 columns per workgroup, 4 lanes per column (16 rows of the block each)
  const int i = blockIdx.x * (kThreads / 4) + (tid & 63);
  const int part = tid >> 6;
  double s = 0.0;
  if (i < k) {
#pragma unroll
    for (int q = 0; q < NB / 4; ++q) {
      const int mm = part * (NB / 4) + q;
      if (mm < kb) s += A[(size_t)(k + mm) * lda + i] * yy[mm];
    }
  }
  __shared__ double red[4][64];
  red[part][tid & 63] = s;
  __syncthreads();
  if (part == 0 && i < k) z[i] -= ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
}

static void enqueue_factor_solve(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y,
                                 int* d_flag);

int chol_factor_solve(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y, int* d_flag) {
  if (n <= 0) return 0;
  const int nblk = (n + NB - 1) / NB;
  if ((size_t)nblk > c->linv_blocks) {
    if (c->exec) (void)hipGraphExecDestroy(c->exec);
    c->exec = nullptr;
    if (c->linv) (void)hipFree(c->linv);
    c->linv = nullptr;
    if (hipMalloc(&c->linv, sizeof(double) * NB * NB * (size_t)nblk) != hipSuccess) return -2;
    c->linv_blocks = nblk;
  }
  const bool same = c->exec && c->g_n == n && c->g_lda == lda && c->g_A == A && c->g_y == y && c->g_flag == d_flag;
  if (!same) {
    if (c->exec) (void)hipGraphExecDestroy(c->exec);
    c->exec = nullptr;
    hipGraph_t g = nullptr;
    if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) return -3;
    enqueue_factor_solve(c, s, n, A, lda, y, d_flag);
    if (hipStreamEndCapture(s, &g) != hipSuccess) return -3;
    const hipError_t e = hipGraphInstantiate(&c->exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) {
      c->exec = nullptr;
      return -3;
    }
    c->g_n = n;
    c->g_lda = lda;
    c->g_A = A;
    c->g_y = y;
    c->g_flag = d_flag;
  }
  return hipGraphLaunch(c->exec, s) == hipSuccess ? 0 : -3;
}

static void enqueue_factor_solve(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y,
                                 int* d_flag) {
  const int nblk = (n + NB - 1) / NB;
  for (int b = 0; b < nblk; ++b) {
    const int k = b * NB, kb = (n - k < NB) ? n - k : NB;
    double* li = c->linv + (size_t)b * NB * NB;
    k_potrf<0><<<1, 64, 0, s>>>(A, lda, k, kb, d_flag);
    k_trinv<<<1, kThreads, 0, s>>>(A, lda, k, kb, li);
    const int r0 = k + kb, r1 = n + 1;  // includes the rhs row n
    k_trsm_inv<<<(r1 - r0 + TR - 1) / TR, kThreads, 0, s>>>(A, lda, k, kb, r0, r1, li);
    const int m = r1 - r0;
    if (m > 1) {
      const int nt = (m + NB - 1) / NB;
      k_syrk_mfma<<<nt * (nt + 1) / 2, kThreads, 0, s>>>(A, lda, r0, m, k, kb);
    }
  }
  double* z = A + (size_t)n * lda;
  for (int b = nblk - 1; b >= 0; --b) {
    const int k = b * NB, kb = (n - k < NB) ? n - k : NB;
    const int grid = k > 0 ? (k + 63) / 64 : 1;
    k_trsv_back<<<grid, kThreads, 0, s>>>(A, lda, k, kb, c->linv + (size_t)b * NB * NB, z, y);
  }
}

}  // namespace dab
