// Operand / result lane layout of v_mfma_f64_4x4x4f64 on gfx950 (one-hot probes).
// out[probe][lane]: probe a < 64: A = e_a, B = lane + 1; probe 64 + b: A = lane + 1, B = e_b
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k_probe(double* out) {
  const int lane = threadIdx.x;
  for (int p = 0; p < 128; ++p) {
    double a, b;
    if (p < 64) { a = lane == p ? 1.0 : 0.0; b = lane + 1.0; }
    else { a = lane + 1.0; b = lane == p - 64 ? 1.0 : 0.0; }
    double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    out[p * 64 + lane] = d;
  }
}
int main() {
  double* d; hipMalloc(&d, 128 * 64 * 8);
  k_probe<<<1, 64>>>(d);
  static double h[128 * 64];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int p = 0; p < 128; ++p) {
    printf("%s %2d:", p < 64 ? "A" : "B", p & 63);
    for (int l = 0; l < 64; ++l) if (h[p * 64 + l] != 0.0) printf(" %d=%g", l, h[p * 64 + l]);
    printf("\n");
  }
  return 0;
}
