// dab_chol.hip — dense Cholesky of the reduced camera system (SURVEY §8a row a7:
// DENSE_SCHUR's "dense Cholesky of S", sfm.cc:67) plus the triangular solves.
//
// S is stored row-major, lower triangle, with the right-hand side appended as row n
// (the augmented matrix [[S, b], [b^T, *]]). Factoring the first n pivots of the
// augmented matrix leaves L in rows 0..n-1 and z = L^-1 b in row n, so the forward
// substitution rides along with the factorisation. Blocked right-looking, NB = 64:
//   potrf + triangular inverse of the 64x64 diagonal block — one workgroup, in LDS
//   panel solve P <- P L_kk^-T as a product with the stored inverse (a small GEMM,
//     every row independent: no sequential substitution on the wide panel)
//   trailing update C -= P P^T — rocBLAS dsyrk (a plain library GEMM)
// Back substitution L^T y = z: one launch per block, y_k = L_kk^-T z_k from the stored
// inverse (a 64x64 matvec) followed by the block-column update of z[0:k].
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include "dab_kernels.h"

namespace dab {

constexpr int NB = 64;

struct CholCtx {
  rocblas_handle h = nullptr;
  double* linv = nullptr;  // [nblk][NB][NB] inverses of the diagonal blocks
  size_t linv_blocks = 0;
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
  if (c->linv) (void)hipFree(c->linv);
  delete c;
}

// Factor A[k:k+kb, k:k+kb] (lower) in place and write its inverse (lower, zero-padded,
// identity beyond kb) to linv[NB][NB].
__global__ __launch_bounds__(256) void k_potrf_inv(double* __restrict__ A, int lda, int k, int kb,
                                                   double* __restrict__ linv, int* __restrict__ flag) {
  __shared__ double a[NB][NB + 1];
  __shared__ double x[NB][NB + 1];
  __shared__ double rdiag[NB];
  const int tid = threadIdx.x;
  for (int idx = tid; idx < NB * NB; idx += blockDim.x) {
    const int i = idx >> 6, j = idx & 63;
    double v;
    if (i < kb && j <= i) v = A[(size_t)(k + i) * lda + k + j];
    else v = (i == j) ? 1.0 : 0.0;
    a[i][j] = v;
  }
  __syncthreads();
  for (int j = 0; j < NB; ++j) {
    const double d = a[j][j];
    const double piv = sqrt(d);
    if (tid == 0 && !(d > 0.0 && isfinite(d))) atomicOr(flag, 1);
    __syncthreads();
    if (tid == j) a[j][j] = piv;
    if (tid > j && tid < NB) a[tid][j] /= piv;
    __syncthreads();
    const int i = tid & 63;
    if (i > j) {
      const double aij = a[i][j];
      for (int l = j + 1 + (tid >> 6); l <= i; l += 4) a[i][l] -= aij * a[l][j];
    }
    __syncthreads();
  }
  if (tid < NB) rdiag[tid] = 1.0 / a[tid][tid];
  __syncthreads();
  // inverse, one column per thread: x = L^-1 e_c
  if (tid < NB) {
    const int c = tid;
    for (int r = 0; r < c; ++r) x[r][c] = 0.0;
    x[c][c] = rdiag[c];
    for (int r = c + 1; r < NB; ++r) {
      double s = 0.0;
      for (int m = c; m < r; ++m) s += a[r][m] * x[m][c];
      x[r][c] = -s * rdiag[r];
    }
  }
  __syncthreads();
  for (int idx = tid; idx < NB * NB; idx += blockDim.x) {
    const int i = idx >> 6, j = idx & 63;
    if (i < kb && j <= i) A[(size_t)(k + i) * lda + k + j] = a[i][j];
    linv[idx] = x[i][j];
  }
}

// rows [r0, r1): A[i, k:k+kb] <- A[i, k:k+kb] Linv^T ; one workgroup per 64 rows
__global__ __launch_bounds__(256) void k_trsm_inv(double* __restrict__ A, int lda, int k, int kb, int r0,
                                                  int r1, const double* __restrict__ linv) {
  __shared__ double P[NB][NB + 1];
  __shared__ double Li[NB][NB + 1];
  const int tid = threadIdx.x;
  const int row0 = r0 + blockIdx.x * NB;
  for (int idx = tid; idx < NB * NB; idx += blockDim.x) {
    const int i = idx >> 6, j = idx & 63;
    Li[i][j] = linv[idx];
    P[i][j] = (row0 + i < r1 && j < kb) ? A[(size_t)(row0 + i) * lda + k + j] : 0.0;
  }
  __syncthreads();
  const int rr = tid >> 2;
  double out[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int j = (tid & 3) + 4 * q;
    double s = 0.0;
    for (int m = 0; m <= j; ++m) s += P[rr][m] * Li[j][m];
    out[q] = s;
  }
  if (row0 + rr < r1) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int j = (tid & 3) + 4 * q;
      if (j < kb) A[(size_t)(row0 + rr) * lda + k + j] = out[q];
    }
  }
}

// back substitution step for block [k, k+kb): y_k = Linv^T z_k, then z[0:k] -= L[k:k+kb, 0:k]^T y_k
__global__ __launch_bounds__(256) void k_trsv_back(const double* __restrict__ A, int lda, int k, int kb,
                                                   const double* __restrict__ linv, double* __restrict__ z,
                                                   double* __restrict__ y) {
  __shared__ double zz[NB];
  __shared__ double yy[NB];
  const int tid = threadIdx.x;
  if (tid < NB) zz[tid] = tid < kb ? z[k + tid] : 0.0;
  __syncthreads();
  if (tid < NB) {
    double s = 0.0;
    for (int m = tid; m < NB; ++m) s += linv[m * NB + tid] * zz[m];
    yy[tid] = s;
  }
  __syncthreads();
  if (blockIdx.x == 0 && tid < kb) y[k + tid] = yy[tid];
  const int i = blockIdx.x * blockDim.x + tid;
  if (i >= k) return;
  double s = 0.0;
  for (int m = 0; m < kb; ++m) s += A[(size_t)(k + m) * lda + i] * yy[m];
  z[i] -= s;
}

int chol_factor_solve(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y, int* d_flag) {
  if (n <= 0) return 0;
  const int nblk = (n + NB - 1) / NB;
  if ((size_t)nblk > c->linv_blocks) {
    if (c->linv) (void)hipFree(c->linv);
    c->linv = nullptr;
    if (hipMalloc(&c->linv, sizeof(double) * NB * NB * (size_t)nblk) != hipSuccess) return -2;
    c->linv_blocks = nblk;
  }
  rocblas_set_stream(c->h, s);
  for (int b = 0; b < nblk; ++b) {
    const int k = b * NB, kb = (n - k < NB) ? n - k : NB;
    double* li = c->linv + (size_t)b * NB * NB;
    k_potrf_inv<<<1, 256, 0, s>>>(A, lda, k, kb, li, d_flag);
    const int r0 = k + kb, r1 = n + 1;  // includes the rhs row n
    k_trsm_inv<<<(r1 - r0 + NB - 1) / NB, 256, 0, s>>>(A, lda, k, kb, r0, r1, li);
    const int m = r1 - r0;
    if (m > 1) {
      const double alpha = -1.0, beta = 1.0;
      rocblas_status st =
          rocblas_dsyrk(c->h, rocblas_fill_upper, rocblas_operation_transpose, m, kb, &alpha,
                        A + (size_t)r0 * lda + k, lda, &beta, A + (size_t)r0 * lda + r0, lda);
      if (st != rocblas_status_success) return -1;
    }
  }
  double* z = A + (size_t)n * lda;
  for (int b = nblk - 1; b >= 0; --b) {
    const int k = b * NB, kb = (n - k < NB) ? n - k : NB;
    const int grid = k > 0 ? (k + 255) / 256 : 1;
    k_trsv_back<<<grid, 256, 0, s>>>(A, lda, k, kb, c->linv + (size_t)b * NB * NB, z, y);
  }
  return 0;
}

}  // namespace dab
