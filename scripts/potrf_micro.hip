// Micro-benchmark of the 64x64 diagonal-block kernel parts (ablation, not product code).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/potrf_micro.hip -o /tmp/potrf_micro
#include "../deeparc-sfm_amd/csrc/dab_chol.hip"

#include <cstdio>
#include <vector>

using namespace dab;

template <int P>
float run(double* A, int lda, double* li, int* flag, hipStream_t s) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int w = 0; w < 5; ++w) k_potrf_inv<P><<<1, kThreads, 0, s>>>(A, lda, 0, 64, li, flag);
  (void)hipEventRecord(e0, s);
  for (int it = 0; it < 200; ++it) k_potrf_inv<P><<<1, kThreads, 0, s>>>(A, lda, 0, 64, li, flag);
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / 200 * 1e3f;
}

int main() {
  const int lda = 72;
  std::vector<double> h(64 * lda, 0.0);
  for (int i = 0; i < 64; ++i) h[i * lda + i] = 1e6;  // stays SPD when re-factored
  double *A, *li;
  int* flag;
  (void)hipMalloc(&A, h.size() * 8);
  (void)hipMalloc(&li, 64 * 64 * 8);
  (void)hipMalloc(&flag, 4);
  (void)hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  printf("load/store only : %8.2f us\n", run<0>(A, lda, li, flag, s));
  printf("factor          : %8.2f us\n", run<1>(A, lda, li, flag, s));
  printf("inverse         : %8.2f us\n", run<2>(A, lda, li, flag, s));
  printf("factor+inverse  : %8.2f us\n", run<3>(A, lda, li, flag, s));
  return 0;
}
