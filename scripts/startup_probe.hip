// Micro-benchmark: how long does the first dependent load of a wave take at kernel start?
// 256 work-groups (one per CU) of 1024 threads (or 256), optionally holding 150 KB of LDS
// like k_eval_bal. Each wave stamps (s_memrealtime, 100 MHz): entry, after a scalar load of
// a per-work-group word (the kernel argument pointer + one dependent load), after a vector
// load indexed by that word, after a second dependent vector load. Back-to-back launches,
// the stamps of the last one are printed as medians relative to the earliest entry.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"

__device__ unsigned long long g_t[256 * 16 * 4];

template <int LDSB>
__global__ __launch_bounds__(1024) void k_probe(const int* __restrict__ beg, const int* __restrict__ idx,
                                                const double* __restrict__ pts, double* out) {
  extern __shared__ double lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const int b = beg[blockIdx.x * 16 + wave];  // uniform: a scalar load
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  const int i = idx[b + lane];
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
  const double x = pts[3 * (size_t)i];
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  const unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
  if (LDSB) lds[threadIdx.x] = x;
  if (x == 1234.5) out[0] = x + (LDSB ? lds[threadIdx.x ^ 1] : 0.0);
  if (lane == 0 && blockIdx.x < 256 && wave < 16) {
    unsigned long long* g = g_t + (blockIdx.x * 16 + wave) * 4;
    g[0] = t0; g[1] = t1; g[2] = t2; g[3] = t3;
  }
}

int main() {
  const int NP = 100000, NE = 1000000;
  std::vector<int> hb(256 * 16), hi(NE);
  for (int k = 0; k < 256 * 16; ++k) hb[k] = (k * 233) % (NE - 64);
  for (int k = 0; k < NE; ++k) hi[k] = (int)((k * 2654435761u) % NP);
  int *db, *di;
  double *dp, *dout;
  hipMalloc(&db, hb.size() * 4); hipMalloc(&di, NE * 4); hipMalloc(&dp, 3 * NP * 8); hipMalloc(&dout, 8);
  hipMemcpy(db, hb.data(), hb.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(di, hi.data(), NE * 4, hipMemcpyHostToDevice);
  hipMemset(dp, 0, 3 * NP * 8);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_probe<1>), hipFuncAttributeMaxDynamicSharedMemorySize,
                            150 * 1024);
  auto run = [&](const char* name, int threads, size_t lds) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int w = 0; w < 20; ++w) {
      if (lds) k_probe<1><<<256, threads, lds>>>(db, di, dp, dout);
      else k_probe<0><<<256, threads, 0>>>(db, di, dp, dout);
    }
    hipEventRecord(e0);
    const int N = 200;
    for (int w = 0; w < N; ++w) {
      if (lds) k_probe<1><<<256, threads, lds>>>(db, di, dp, dout);
      else k_probe<0><<<256, threads, 0>>>(db, di, dp, dout);
    }
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    if (hipGetLastError() != hipSuccess) { printf("%s: launch failed\n", name); return; }
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> t(256 * 16 * 4);
    hipMemcpyFromSymbol(t.data(), HIP_SYMBOL(g_t), t.size() * 8);
    const int nw = threads / 64;
    unsigned long long tmin = ~0ull;
    for (int b = 0; b < 256; ++b)
      for (int w = 0; w < nw; ++w) tmin = std::min(tmin, t[(b * 16 + w) * 4]);
    std::vector<double> d[4];
    for (int b = 0; b < 256; ++b)
      for (int w = 0; w < nw; ++w)
        for (int k = 0; k < 4; ++k) d[k].push_back((t[(b * 16 + w) * 4 + k] - tmin) * 0.01);
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    auto mx = [](std::vector<double> v) { return *std::max_element(v.begin(), v.end()); };
    printf("%-26s per launch %6.2f us | entry %5.2f (max %5.2f)  scalar %5.2f  index %5.2f  gather %5.2f (max %5.2f) us\n",
           name, 1e3 * ms / N, med(d[0]), mx(d[0]), med(d[1]), med(d[2]), med(d[3]), mx(d[3]));
  };
  run("1024 thr, no LDS", 1024, 0);
  run("1024 thr, 150 KB LDS", 1024, 150 * 1024);
  run("256 thr, no LDS", 256, 0);
  run("256 thr, 150 KB LDS", 256, 150 * 1024);
  return 0;
}
