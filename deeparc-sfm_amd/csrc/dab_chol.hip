// dab_chol.hip — dense Cholesky of the reduced camera system (SURVEY §8a row a7:
// DENSE_SCHUR's "dense Cholesky of S", sfm.cc:67) plus the triangular solves.
//
// S is stored row-major, lower triangle, with the right-hand side appended as row n
// (the augmented matrix [[S, b], [b^T, *]]). Factoring the first n pivots of the
// augmented matrix leaves L in rows 0..n-1 and z = L^-1 b in row n, so the forward
// substitution rides along with the factorisation. Blocked right-looking, NB = 64:
//   potrf of the 64x64 diagonal block  — one workgroup, LDS-resident (hand-written)
//   panel TRSM of the rows below       — one row per lane, L_kk in LDS (hand-written)
//   trailing update C -= P P^T          — rocBLAS dsyrk (a plain library GEMM)
// Back substitution L^T y = z: one launch per 64-block, each workgroup re-solves the
// 64x64 triangle from L2 and applies the block column update to 256 entries of z.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include "dab_kernels.h"

namespace dab {

constexpr int NB = 64;

struct CholCtx {
  rocblas_handle h = nullptr;
};

CholCtx* chol_create() {
  CholCtx* c = new CholCtx();
  if (rocblas_create_handle(&c->h) != rocblas_status_success) {
    delete c;
    return nullptr;
  }
  rocblas_set_pointer_mode(c->h, rocblas_pointer_mode_host);
  return c;
}
void chol_destroy(CholCtx* c) {
  if (!c) return;
  if (c->h) rocblas_destroy_handle(c->h);
  delete c;
}

// factor A[k:k+kb, k:k+kb] (lower) in place
__global__ __launch_bounds__(256) void k_potrf_diag(double* __restrict__ A, int lda, int k, int kb,
                                                    int* __restrict__ flag) {
  __shared__ double a[NB][NB + 1];
  const int tid = threadIdx.x;
  for (int idx = tid; idx < NB * NB; idx += blockDim.x) {
    const int i = idx / NB, j = idx - NB * (idx / NB);
    a[i][j] = (i < kb && j <= i) ? A[(size_t)(k + i) * lda + k + j] : 0.0;
  }
  __syncthreads();
  for (int j = 0; j < kb; ++j) {
    if (tid == 0) {
      const double d = a[j][j];
      if (!(d > 0.0) || !isfinite(d)) atomicOr(flag, 1);
      a[j][j] = sqrt(d);
    }
    __syncthreads();
    const double piv = a[j][j];
    for (int i = j + 1 + tid; i < kb; i += blockDim.x) a[i][j] /= piv;
    __syncthreads();
    const int m = kb - j - 1;  // trailing size
    for (int idx = tid; idx < m * m; idx += blockDim.x) {
      const int i = j + 1 + idx / m, l = j + 1 + (idx - m * (idx / m));
      if (l <= i) a[i][l] -= a[i][j] * a[l][j];
    }
    __syncthreads();
  }
  for (int idx = tid; idx < NB * NB; idx += blockDim.x) {
    const int i = idx / NB, j = idx - NB * (idx / NB);
    if (i < kb && j <= i) A[(size_t)(k + i) * lda + k + j] = a[i][j];
  }
}

// rows [r0, r1): A[i, k:k+kb] <- A[i, k:k+kb] L_kk^-T
__global__ __launch_bounds__(256) void k_trsm_panel(double* __restrict__ A, int lda, int k, int kb,
                                                    int r0, int r1) {
  __shared__ double L[NB][NB + 1];
  for (int idx = threadIdx.x; idx < NB * NB; idx += blockDim.x) {
    const int i = idx / NB, j = idx - NB * (idx / NB);
    double v = 0.0;
    if (i < kb && j <= i) v = A[(size_t)(k + i) * lda + k + j];
    else if (i == j) v = 1.0;
    L[i][j] = v;
  }
  __syncthreads();
  const int i = r0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= r1) return;
  double* row = A + (size_t)i * lda + k;
  double x[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) x[j] = (j < kb) ? row[j] : 0.0;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    double s = x[j];
#pragma unroll
    for (int m = 0; m < j; ++m) s -= x[m] * L[j][m];
    x[j] = s / L[j][j];
  }
#pragma unroll
  for (int j = 0; j < NB; ++j)
    if (j < kb) row[j] = x[j];
}

// back substitution step for block [k, k+kb): y_k = L_kk^-T z_k, then z[0:k] -= L[k:k+kb, 0:k]^T y_k
__global__ __launch_bounds__(256) void k_trsv_back(const double* __restrict__ A, int lda, int n, int k,
                                                   int kb, double* __restrict__ z, double* __restrict__ y) {
  __shared__ double L[NB][NB + 1];
  __shared__ double zz[NB];
  for (int idx = threadIdx.x; idx < NB * NB; idx += blockDim.x) {
    const int i = idx / NB, j = idx - NB * (idx / NB);
    L[i][j] = (i < kb && j <= i) ? A[(size_t)(k + i) * lda + k + j] : 0.0;
  }
  if (threadIdx.x < NB) zz[threadIdx.x] = threadIdx.x < kb ? z[k + threadIdx.x] : 0.0;
  __syncthreads();
  // L_kk^T y = zz, upper-triangular solve, descending
  for (int j = kb - 1; j >= 0; --j) {
    if (threadIdx.x == 0) zz[j] = zz[j] / L[j][j];
    __syncthreads();
    const double yj = zz[j];
    if (threadIdx.x < j) zz[threadIdx.x] -= L[j][threadIdx.x] * yj;
    __syncthreads();
  }
  if (blockIdx.x == 0 && threadIdx.x < kb) y[k + threadIdx.x] = zz[threadIdx.x];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  double s = 0.0;
  for (int m = 0; m < kb; ++m) s += A[(size_t)(k + m) * lda + i] * zz[m];
  z[i] -= s;
}

int chol_factor_solve(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y, int* d_flag) {
  if (n <= 0) return 0;
  rocblas_set_stream(c->h, s);
  for (int k = 0; k < n; k += NB) {
    const int kb = (n - k < NB) ? n - k : NB;
    k_potrf_diag<<<1, 256, 0, s>>>(A, lda, k, kb, d_flag);
    const int r0 = k + kb, r1 = n + 1;  // includes the rhs row n
    if (r1 > r0) {
      k_trsm_panel<<<(r1 - r0 + 255) / 256, 256, 0, s>>>(A, lda, k, kb, r0, r1);
      const int m = r1 - r0;
      const double alpha = -1.0, beta = 1.0;
      rocblas_status st =
          rocblas_dsyrk(c->h, rocblas_fill_upper, rocblas_operation_transpose, m, kb, &alpha,
                        A + (size_t)r0 * lda + k, lda, &beta, A + (size_t)r0 * lda + r0, lda);
      if (st != rocblas_status_success) return -1;
    }
  }
  // z = row n; back substitution (z is updated in place)
  double* z = A + (size_t)n * lda;
  const int nblk = (n + NB - 1) / NB;
  for (int b = nblk - 1; b >= 0; --b) {
    const int k = b * NB, kb = (n - k < NB) ? n - k : NB;
    const int grid = k > 0 ? (k + 255) / 256 : 1;
    k_trsv_back<<<grid, 256, 0, s>>>(A, lda, n, k, kb, z, y);
  }
  return 0;
}

}  // namespace dab
