// Micro-benchmark + cross-check of the panel kernel (not product code): k_panel on a random
// SPD 64x64 block (L_kk against a CPU Cholesky) and on a 6000-row panel, with the phase
// profile of one launch (wall clock, 100 MHz).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/potrf_micro.hip -o scripts/potrf_micro
// (factor16 as shipped; the round-5 form and the DPP64-fmac variant are in
// scripts/experiments/chol_bulk_lds_dma_f16_asm.patch)
#define DAB_CHOL_PROFILE
#include "../deeparc-sfm_amd/csrc/dab_chol.hip"

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

using namespace dab;

// the solver's process-wide stream cache, which dab_chol.hip links against
namespace dab {
hipStream_t stream_take(int) {
  hipStream_t s = nullptr;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  return s;
}
void stream_give(int, hipStream_t s) { (void)hipStreamDestroy(s); }
int set_error(int code, const std::string& msg) {
  fprintf(stderr, "%s\n", msg.c_str());
  return code;
}
}  // namespace dab

__global__ void k_empty() {}

int main() {
  const int lda = 72, n = 64;
  std::mt19937_64 rng(3);
  std::normal_distribution<double> nd;
  std::vector<double> G(64 * 64), h(65 * lda, 0.0);
  for (auto& v : G) v = nd(rng);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = (i == j) ? 64.0 : 0.0;
      for (int k = 0; k < 64; ++k) s += G[i * 64 + k] * G[j * 64 + k];
      h[i * lda + j] = s;
    }
  for (int j = 0; j < n; ++j) h[64 * lda + j] = nd(rng);  // one panel row (the rhs)
  // CPU reference: L and z = L^-1 b
  std::vector<double> Lr(64 * 64, 0.0), zr(64);
  for (int j = 0; j < 64; ++j) {
    double d = h[j * lda + j];
    for (int m = 0; m < j; ++m) d -= Lr[j * 64 + m] * Lr[j * 64 + m];
    Lr[j * 64 + j] = std::sqrt(d);
    for (int i = j + 1; i < 64; ++i) {
      double s = h[i * lda + j];
      for (int m = 0; m < j; ++m) s -= Lr[i * 64 + m] * Lr[j * 64 + m];
      Lr[i * 64 + j] = s / Lr[j * 64 + j];
    }
  }
  for (int i = 0; i < 64; ++i) {
    double s = h[64 * lda + i];
    for (int m = 0; m < i; ++m) s -= Lr[i * 64 + m] * zr[m];
    zr[i] = s / Lr[i * 64 + i];
  }
  double *A, *blk, *Big;
  int* flag;
  (void)hipMalloc(&A, h.size() * 8);
  (void)hipMalloc(&blk, kBlk * 8 * 100);
  (void)hipMalloc(&flag, 4);
  (void)hipMalloc(&Big, sizeof(double) * 6008 * 6001);
  (void)hipMemset(Big, 0, sizeof(double) * 6008 * 6001);
  (void)hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemset(flag, 0, 4);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  k_panel<<<1, kThreads, 0, s>>>(A, lda, 0, 64, 64, 65, blk, flag, 0);
  (void)hipStreamSynchronize(s);
  std::vector<double> hb(kBlk), ha(h.size());
  (void)hipMemcpy(hb.data(), blk, kBlk * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(ha.data(), A, h.size() * 8, hipMemcpyDeviceToHost);
  double dl = 0, ml = 0, dz = 0, mz = 0;
  for (int i = 0; i < 64; ++i) {
    for (int j = 0; j <= i; ++j) {
      dl = std::max(dl, std::fabs(hb[1024 + i * 64 + j] - Lr[i * 64 + j]));
      ml = std::max(ml, std::fabs(Lr[i * 64 + j]));
    }
    dz = std::max(dz, std::fabs(ha[64 * lda + i] - zr[i]));
    mz = std::max(mz, std::fabs(zr[i]));
  }
  int fl = 0;
  (void)hipMemcpy(&fl, flag, 4, hipMemcpyDeviceToHost);
  printf("k_panel vs CPU: max |dL|/max|L| %.2e  max |dz|/max|z| %.2e  flag %d\n", dl / ml, dz / mz, fl);

  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[] = {"empty", "panel (diag + 1 row)", "panel (6000 rows)"};
  for (int var = 0; var < 3; ++var) {
    float best = 1e9f;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0, s);
      for (int it = 0; it < 100; ++it) {
        if (var == 0) k_empty<<<1, 64, 0, s>>>();
        if (var == 1) k_panel<<<1, kThreads, 0, s>>>(A, lda, 0, 64, 64, 65, blk, flag, 0);
        if (var == 2) k_panel<<<94, kThreads, 0, s>>>(Big, 6008, 0, 64, 64, 6000, blk, flag, 0);
      }
      (void)hipEventRecord(e1, s);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      best = std::min(best, ms / 100 * 1e3f);
    }
    printf("%-22s %8.2f us per launch\n", names[var], best);
    if (var > 0) {  // phase profile of the last (warm) launch
      long long pr[16];
      (void)hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_prof), sizeof(pr));
      const char* ph[] = {"load", "sync", "f16 p0", "stage p0", "f16 p1", "stage p1", "f16 p2", "stage p2", "f16 p3", "-",
                          "P solve"};
      long long prev = pr[0];
      for (int i = 1; i <= 10; ++i) {
        if (i == 9) continue;
        printf("    %-9s %6.2f us\n", ph[i], (pr[i] - prev) * 0.01);
        prev = pr[i];
      }
    }
  }
  return 0;
}
