// Dense Cholesky micro-benchmark (GPU box): libdab's factor+solve of the augmented
// row-major lower matrix against rocSOLVER dpotrf + dpotrs on the same SPD matrix.
// rocSOLVER is only a yardstick here; the product path never calls it.
// Build: hipcc -O2 -std=c++17 scripts/chol_micro.cpp -Ideeparc-sfm_amd/csrc -Ldeeparc-sfm_amd -ldab
//        -lrocsolver -lrocblas -Wl,-rpath,$PWD/deeparc-sfm_amd -o scripts/chol_micro
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

namespace dab {
struct CholCtx;
CholCtx* chol_create();
void chol_destroy(CholCtx*);
int chol_factor_solve(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y, int* d_flag);
}  // namespace dab

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 5994;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  int lds = ((n + 1 + 7) / 8) * 8;
  if (lds % 512 == 0) lds += 8;
  // SPD: S = G G^T / n + I with G random (condition number ~ 5)
  std::mt19937_64 rng(7);
  std::normal_distribution<double> nd;
  std::vector<double> G((size_t)n * 64);
  for (auto& v : G) v = nd(rng);
  std::vector<double> S((size_t)n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = 0.0;
      for (int k = 0; k < 64; ++k) s += G[(size_t)i * 64 + k] * G[(size_t)j * 64 + k];
      s = s / 64.0 + (i == j ? 1.0 : 0.0) + 0.01 * std::cos(0.001 * (i - j));
      S[(size_t)i * n + j] = S[(size_t)j * n + i] = s;
    }
  std::vector<double> b(n);
  for (auto& v : b) v = nd(rng);
  // augmented row-major lower copy for libdab
  std::vector<double> Aug((size_t)(n + 1) * lds, 0.0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) Aug[(size_t)i * lds + j] = S[(size_t)i * n + j];
  for (int j = 0; j < n; ++j) Aug[(size_t)n * lds + j] = b[j];

  hipStream_t s;
  CK(hipStreamCreate(&s));
  double *dAug, *dA0, *dy;
  int* dflag;
  CK(hipMalloc(&dAug, sizeof(double) * Aug.size()));
  CK(hipMalloc(&dA0, sizeof(double) * Aug.size()));
  CK(hipMalloc(&dy, sizeof(double) * n));
  CK(hipMalloc(&dflag, sizeof(int)));
  CK(hipMemcpy(dA0, Aug.data(), sizeof(double) * Aug.size(), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  dab::CholCtx* c = dab::chol_create();
  float best = 1e30f, sum = 0.f;
  std::vector<double> y(n);
  for (int r = 0; r < reps + 1; ++r) {
    CK(hipMemcpyAsync(dAug, dA0, sizeof(double) * Aug.size(), hipMemcpyDeviceToDevice, s));
    CK(hipMemsetAsync(dflag, 0, sizeof(int), s));
    if (r == 0) {  // first call captures the graph
      if (dab::chol_factor_solve(c, s, n, dAug, lds, dy, dflag)) return 2;
      CK(hipStreamSynchronize(s));
      continue;
    }
    CK(hipEventRecord(e0, s));
    if (dab::chol_factor_solve(c, s, n, dAug, lds, dy, dflag)) return 2;
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, ms);
    sum += ms;
  }
  int flag = 0;
  CK(hipMemcpy(&flag, dflag, sizeof(int), hipMemcpyDeviceToHost));
  CK(hipMemcpy(y.data(), dy, sizeof(double) * n, hipMemcpyDeviceToHost));
  double rn = 0.0, bn = 0.0;
  for (int i = 0; i < n; ++i) {
    double t = -b[i];
    for (int j = 0; j < n; ++j) t += S[(size_t)i * n + j] * y[j];
    rn += t * t;
    bn += b[i] * b[i];
  }
  const double gf = (double)n * n * n / 3.0 * 1e-9;
  printf("libdab   n=%d: factor+solve best %.3f ms mean %.3f ms (%.2f TFLOP/s), flag %d, |Sx-b|/|b| %.2e\n", n, best,
         sum / reps, gf / best, flag, std::sqrt(rn / bn));
  dab::chol_destroy(c);

  // rocSOLVER: column-major lower == row-major upper; use the full symmetric matrix
  rocblas_handle rb;
  rocblas_create_handle(&rb);
  rocblas_set_stream(rb, s);
  double *dS, *dS0, *db;
  rocblas_int* dinfo;
  CK(hipMalloc(&dS, sizeof(double) * S.size()));
  CK(hipMalloc(&dS0, sizeof(double) * S.size()));
  CK(hipMalloc(&db, sizeof(double) * n));
  CK(hipMalloc(&dinfo, sizeof(rocblas_int)));
  CK(hipMemcpy(dS0, S.data(), sizeof(double) * S.size(), hipMemcpyHostToDevice));
  best = 1e30f;
  sum = 0.f;
  for (int r = 0; r < reps + 1; ++r) {
    CK(hipMemcpyAsync(dS, dS0, sizeof(double) * S.size(), hipMemcpyDeviceToDevice, s));
    CK(hipMemcpyAsync(db, b.data(), sizeof(double) * n, hipMemcpyHostToDevice, s));
    CK(hipEventRecord(e0, s));
    rocsolver_dpotrf(rb, rocblas_fill_lower, n, dS, n, dinfo);
    rocsolver_dpotrs(rb, rocblas_fill_lower, n, 1, dS, n, db, n);
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r > 0) {
      best = std::min(best, ms);
      sum += ms;
    }
  }
  printf("rocsolver n=%d: potrf+potrs best %.3f ms mean %.3f ms (%.2f TFLOP/s)\n", n, best, sum / reps, gf / best);
  rocblas_destroy_handle(rb);
  return 0;
}
