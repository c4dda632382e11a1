// Accuracy of v_rsq_f64 and of one / two Newton steps on it, against a correctly rounded
// 1/sqrt (long double on the host), over 2^20 random pivots in [1e-3, 1e9) (the dense
// Cholesky's factor16 takes 1/sqrt(d) of every pivot: rsq + two Newton steps).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/rsq_probe.hip -o scripts/rsq_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

__global__ void k_rsq(const double* d, double* o0, double* o1, double* o2, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = d[i];
  double y = __builtin_amdgcn_rsq(x);
  o0[i] = y;
  y = y * fma(-0.5 * x * y, y, 1.5);
  o1[i] = y;
  y = y * fma(-0.5 * x * y, y, 1.5);
  o2[i] = y;
}

int main() {
  const int n = 1 << 20;
  std::mt19937_64 rng(5);
  std::uniform_real_distribution<double> u(std::log(1e-3), std::log(1e9));
  std::vector<double> h(n);
  for (auto& v : h) v = std::exp(u(rng));
  double *d, *o0, *o1, *o2;
  (void)hipMalloc(&d, n * 8);
  (void)hipMalloc(&o0, n * 8);
  (void)hipMalloc(&o1, n * 8);
  (void)hipMalloc(&o2, n * 8);
  (void)hipMemcpy(d, h.data(), n * 8, hipMemcpyHostToDevice);
  k_rsq<<<(n + 255) / 256, 256>>>(d, o0, o1, o2, n);
  std::vector<double> r0(n), r1(n), r2(n);
  (void)hipMemcpy(r0.data(), o0, n * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(r1.data(), o1, n * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(r2.data(), o2, n * 8, hipMemcpyDeviceToHost);
  double e[3] = {0, 0, 0};
  long long exact[3] = {0, 0, 0};
  for (int i = 0; i < n; ++i) {
    const long double ref = 1.0L / std::sqrt((long double)h[i]);
    const double cr = (double)ref;  // correctly rounded (to long double precision first)
    const double* r[3] = {&r0[i], &r1[i], &r2[i]};
    for (int k = 0; k < 3; ++k) {
      const double ulp = std::nextafter(cr, 1e300) - cr;
      e[k] = std::fmax(e[k], std::fabs((long double)*r[k] - ref) / ulp);
      exact[k] += *r[k] == cr;
    }
  }
  printf("v_rsq_f64 alone: max %.3g ulp, %.4f exact\n", e[0], exact[0] / (double)n);
  printf("+1 Newton step : max %.3g ulp, %.4f exact\n", e[1], exact[1] / (double)n);
  printf("+2 Newton steps: max %.3g ulp, %.4f exact\n", e[2], exact[2] / (double)n);
  return 0;
}
