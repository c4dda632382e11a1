// Standalone check of k_eval_bal's in-launch table protocol (claim / produce / done / wait)
// with the same grid shape (256 x 1024, one work-group per CU): prints each work-group's
// wait time and the counters. hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__device__ __forceinline__ int xcc() { return __builtin_amdgcn_s_getreg(20 | (3 << 11)) & 7; }

__global__ __launch_bounds__(1024) void k_proto(unsigned* sync, double* tab, int E, unsigned* out, int par) {
  __shared__ unsigned ready;
  __shared__ double big[18000];  // ~144 KB: one work-group per CU, as k_eval_bal
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) ready = 0u;
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < 256; i += blockDim.x) sync[(par ^ 1) * 256 + i] = 0u;
  __syncthreads();
  const int x = xcc();
  unsigned* ctr = sync + (par * 8 + x) * 32;
  const unsigned nch = (E + 63) / 64;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned claims = 0;
  if (wave == 0) {
    for (;;) {
      unsigned o = 0;
      if (lane == 0) o = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      o = __builtin_amdgcn_readfirstlane(o);
      if (o >= nch) break;
      ++claims;
      const int e = (int)o * 64 + lane;
      if (e < E) tab[((size_t)x * E + e) * 16] = (double)e;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (claims > 100000) break;
    }
    if (lane == 0) {
      while (__hip_atomic_load(ctr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < nch) {
        __builtin_amdgcn_s_sleep(2);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) break;
      }
      __hip_atomic_store(&ready, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  while (__hip_atomic_load(&ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u) {
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > 5000000ull) break;
  }
  big[threadIdx.x] = 1.0;
  if (threadIdx.x == 0) {
    out[4 * blockIdx.x] = x;
    out[4 * blockIdx.x + 1] = claims;
    out[4 * blockIdx.x + 2] = (unsigned)(__builtin_amdgcn_s_memrealtime() - t0);
    out[4 * blockIdx.x + 3] = (unsigned)big[5];
  }
}

int main() {
  const int E = 1000;
  unsigned *sync, *out;
  double* tab;
  hipMalloc(&sync, 512 * 4);
  hipMalloc(&out, 256 * 4 * 4);
  hipMalloc(&tab, 8 * E * 16 * 8);
  hipMemset(sync, 0, 512 * 4);
  for (int it = 0; it < 4; ++it) {
    k_proto<<<256, 1024>>>(sync, tab, E, out, it & 1);
    if (hipDeviceSynchronize() != hipSuccess) {
      std::printf("launch %d failed\n", it);
      return 2;
    }
    std::vector<unsigned> h(1024), s(512);
    hipMemcpy(h.data(), out, 4096, hipMemcpyDeviceToHost);
    hipMemcpy(s.data(), sync, 2048, hipMemcpyDeviceToHost);
    unsigned mx = 0, cl = 0;
    for (int b = 0; b < 256; ++b) {
      mx = std::max(mx, h[4 * b + 2]);
      cl += h[4 * b + 1];
    }
    std::printf("launch %d: claims %u, slowest wait %.2f us; counters (set %d):", it, cl, mx * 0.01, it & 1);
    for (int x = 0; x < 8; ++x) std::printf(" %u/%u", s[(it & 1) * 256 + x * 32], s[(it & 1) * 256 + x * 32 + 1]);
    std::printf("\n");
  }
  return 0;
}
