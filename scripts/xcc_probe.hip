// Which XCD runs each work-group (HW_REG_XCC_ID), 256 work-groups of 64 threads: prints the
// id histogram and whether blockIdx % 8 predicts it. hipcc --offload-arch=gfx950 -O2
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_xcc(int* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = __builtin_amdgcn_s_getreg(20 | (3 << 11));
}

int main() {
  int* d = nullptr;
  if (hipMalloc(&d, 256 * sizeof(int)) != hipSuccess) return 1;
  k_xcc<<<256, 64>>>(d);
  if (hipDeviceSynchronize() != hipSuccess) {
    std::printf("kernel failed\n");
    return 2;
  }
  int h[256];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 3;
  int hist[16] = {0};
  bool mod8 = true;
  for (int b = 0; b < 256; ++b) {
    hist[h[b] & 15]++;
    if ((h[b] & 7) != (h[b % 8] & 7)) mod8 = false;
  }
  std::printf("xcc ids of blocks 0-15:");
  for (int b = 0; b < 16; ++b) std::printf(" %d", h[b]);
  std::printf("\nhistogram:");
  for (int i = 0; i < 16; ++i) std::printf(" %d", hist[i]);
  std::printf("\nblockIdx %% 8 groups share an id: %s\n", mod8 ? "yes" : "no");
  return 0;
}
