// Calibration: how fast can one launch stream the point kernel's inputs on MI355X?
// Reads N slots of (int4 idx, double2 xy) = 32 B/slot (the SELL observation streams) and
// writes one partial per work-group. Reports the average kernel time per grid shape.
// build: hipcc -O3 --offload-arch=gfx950 scripts/stream_micro.hip -o scripts/stream_micro
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

template <int UNROLL>
__global__ void k_stream(int n, const int4* __restrict__ idx, const double2* __restrict__ xy,
                         double* __restrict__ part) {
  double a = 0.0;
  const int stride = gridDim.x * blockDim.x;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
    int4 d[UNROLL];
    double2 x[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      d[u] = idx[i + u * stride];
      x[u] = xy[i + u * stride];
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) a += x[u].x + x[u].y + d[u].y + d[u].w;
  }
  for (; i < n; i += stride) {
    const int4 d = idx[i];
    const double2 x = xy[i];
    a += x.x + x.y + d.y + d.w;
  }
  // one partial per wave (no block-level tail)
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
  if ((threadIdx.x & 63) == 0) part[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = a;
}

template <int LDSKB>
__global__ void k_empty(double* part) {
  __shared__ double big[LDSKB * 128];
  big[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) part[0] = big[5];
}
template <int LDSKB>
float run_empty(double* part, int grid, int block, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  k_empty<LDSKB><<<grid, block>>>(part);
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) k_empty<LDSKB><<<grid, block>>>(part);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps * 1e3f;
}

template <int U>
float run(int n, const int4* idx, const double2* xy, double* part, int grid, int block, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int r = 0; r < 5; ++r) k_stream<U><<<grid, block>>>(n, idx, xy, part);
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) k_stream<U><<<grid, block>>>(n, idx, xy, part);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps * 1e3f;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 1000000;
  int4* idx;
  double2* xy;
  double* part;
  CK(hipMalloc(&idx, sizeof(int4) * n));
  CK(hipMalloc(&xy, sizeof(double2) * n));
  CK(hipMalloc(&part, sizeof(double) * (1 << 20)));
  CK(hipMemset(idx, 0, sizeof(int4) * n));
  CK(hipMemset(xy, 0, sizeof(double2) * n));
  const double mb = 32.0 * n / 1e6;
  struct Shape {
    int grid, block;
  } shapes[] = {{256, 1024}, {512, 1024}, {1024, 256}, {2048, 256}, {4096, 256}, {(n + 255) / 256, 256}};
  const int reps = 200;
  for (auto sh : shapes) {
    const float u1 = run<1>(n, idx, xy, part, sh.grid, sh.block, reps);
    const float u4 = run<4>(n, idx, xy, part, sh.grid, sh.block, reps);
    printf("n=%d (%.1f MB) grid %5d x %4d: unroll1 %.2f us (%.0f GB/s), unroll4 %.2f us (%.0f GB/s)\n", n, mb,
           sh.grid, sh.block, u1, mb * 1e3 / u1, u4, mb * 1e3 / u4);
  }
  const int eg[][2] = {{256, 1024}, {1024, 256}, {4096, 256}, {256, 256}};
  for (auto e : eg)
    printf("empty %4d x %4d: 1 KB LDS %.2f us, 150 KB LDS %.2f us\n", e[0], e[1], run_empty<1>(part, e[0], e[1], reps),
           run_empty<150>(part, e[0], e[1], reps));
  // the same launches captured once into a graph and replayed
  for (auto e : eg) {
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int r = 0; r < reps; ++r) k_stream<1><<<e[0], e[1], 0, st>>>(n, idx, xy, part);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const float us_stream = run<1>(n, idx, xy, part, e[0], e[1], reps);
    printf("stream kernel %4d x %4d: graph %.2f us/launch, stream %.2f us/launch\n", e[0], e[1], ms / reps * 1e3f,
           us_stream);
  }
  return 0;
}
