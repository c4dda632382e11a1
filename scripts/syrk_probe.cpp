// rocBLAS dsyrk / dgemm at the Cholesky's bulk-update shapes (rank-128 update of the
// trailing m x m block, C3's n = 5994): achieved TFLOP/s, to compare with k_syrk_big.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <cstdio>
#include <vector>

int main() {
  rocblas_handle h;
  rocblas_create_handle(&h);
  const int lda = 6016, n = 5994;
  double *A;
  (void)hipMalloc(&A, sizeof(double) * (size_t)lda * (n + 1));
  (void)hipMemset(A, 0, sizeof(double) * (size_t)lda * (n + 1));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const double alpha = -1.0, beta = 1.0;
  for (int m : {5800, 4000, 2000, 800}) {
    for (int k : {64, 128, 256}) {
      const double* X = A + 0;            // k x m (column-major view), ld = lda
      double* C = A + (size_t)lda * 256;  // m x m
      for (int w = 0; w < 3; ++w)
        rocblas_dsyrk(h, rocblas_fill_upper, rocblas_operation_transpose, m, k, &alpha, X, lda, &beta, C, lda);
      (void)hipEventRecord(e0);
      const int R = 10;
      for (int w = 0; w < R; ++w)
        rocblas_dsyrk(h, rocblas_fill_upper, rocblas_operation_transpose, m, k, &alpha, X, lda, &beta, C, lda);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double us = 1e3 * ms / R, fl = (double)m * m * k;  // n^2 k flops for the triangle (2 x half)
      printf("dsyrk m=%5d k=%3d: %8.1f us  %6.2f TFLOP/s\n", m, k, us, fl / (us * 1e-6) / 1e12);
    }
  }
  rocblas_destroy_handle(h);
  return 0;
}
