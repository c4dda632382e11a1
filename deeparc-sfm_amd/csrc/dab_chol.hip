// dab_chol.hip — dense Cholesky of the reduced camera system (SURVEY §8a row a7:
// DENSE_SCHUR's "dense Cholesky of S", sfm.cc:67) plus the triangular solves.
//
// S is stored row-major, lower triangle, with the right-hand side appended as row n
// (the augmented matrix [[S, b], [b^T, *]]). Factoring the first n pivots of the
// augmented matrix leaves L in rows 0..n-1 and z = L^-1 b in row n, so the forward
// substitution rides along with the factorisation. Blocked right-looking, NB = 64, panels
// in pairs (the chain on one stream, the rank-128 bulk update of each pair on a second):
//   k_panel      the first panel step: every work-group factors the 64x64 diagonal block
//                (16x16 sub-blocks in registers, rank-16 updates and the panel solve on
//                fp64 MFMA) and solves its own 64 rows below it with the 16x16 inverses
//   k_syrk_mfma  the column update in front of each later panel (fp64 MFMA, 4 waves x 32x32
//                quadrants): its diagonal-tile work-group factors the block and publishes
//                L_kk and the inverses (ready flag); the other work-groups wait for it and
//                solve their tile's panel rows, so one launch per block carries the chain
//   k_syrk_big   the bulk trailing update of a panel pair on 128x128 super-tiles
//   k_trsv_back_flow  L^T y = z as a dataflow over the blocks (owners keep z in LDS,
//                per-block ready flags, no grid barrier)
// The whole sequence is captured once into a hipGraph (two streams) and replayed;
// DAB_CHOL_V1=1 keeps the round-1 per-step schedule.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dab_devmem.h"
#include "dab_kernels.h"
#include "dab_wave.h"

namespace dab {

constexpr int NB = 64;
constexpr int kThreads = 256;
constexpr int LDP = 66;  // padded LDS row stride (doubles): conflict-free fragment reads
constexpr int kBlk = 1024 + NB * NB;

typedef double dbl4 __attribute__((ext_vector_type(4)));

struct CholCtx {
  Dev mem{"Cholesky scratch"};  // every device buffer below (guarded like the problem's)
  double* blk = nullptr;  // per block column: D [4][16][16] (inverses of the 16x16 diagonal
                          // blocks), then L_kk [64][64]; stride kBlk

  hipStream_t side = nullptr;                     // bulk trailing updates (captured into the graph)
  int device = 0;
  std::vector<hipEvent_t> ev_panel, ev_bulk, ev_strip;  // per block column
  size_t nblk_alloc = 0;
  // the ~5 x n/64 dependent launches are captured once per (n, buffers) and replayed
  hipGraphExec_t exec = nullptr;
  int g_n = -1, g_lda = -1;
  const void *g_A = nullptr, *g_y = nullptr, *g_flag = nullptr;
  int bulk_grid = 0;  // work-groups of the persistent bulk update (0: one per tile)
  int ncu = 256;
  unsigned* bar = nullptr;  // grid-barrier counter of k_trsv_back_all (zeroed per solve)
  bool back_flow = true;      // DAB_CHOL_BACK_FLOW=0: the grid-barrier back substitution
  bool prefactor = true;      // DAB_CHOL_PREFACTOR=0: every panel work-group factors the diagonal block
  bool nograph = false;       // DAB_CHOL_NOGRAPH=1: launch directly instead of the captured graph (traces)
  int graph_min = 16;         // DAB_CHOL_GRAPH_MIN: fewest blocks that use the captured graph
  bool serial = false;        // DAB_CHOL_SERIAL=1: the bulk updates on the chain stream (debugging)
  bool fuse_panel = true;     // DAB_CHOL_FUSE_PANEL=0: the panel step as its own launch after the column update
  unsigned* pready = nullptr; // per block: L_kk published by the fused column update (zeroed per factorisation)
  int group = 2;            // DAB_CHOL_GROUP: panels per bulk trailing update (2: pairs)
  bool strip = true;        // DAB_CHOL_STRIP=0: the bulk's first block column inside the bulk launch
                            // (round 4's schedule) instead of a launch of its own
  bool v1 = false;          // DAB_CHOL_V1=1: the per-step schedule (one bulk update per panel, one
                            // back-substitution launch per block)
};

CholCtx* chol_create() {
  CholCtx* c = new CholCtx();
  int ncu = 256;
  hipDeviceProp_t prop;
  int dev = 0;
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0)
    ncu = prop.multiProcessorCount;
  // two 512-thread bulk work-groups per CU, 32 CUs left for the panel chain (measured at
  // n = 5994: 6.74 ms against 6.88-6.93 ms for one per CU or all CUs)
  c->bulk_grid = std::max(1, 2 * ncu - 64);
  c->ncu = ncu;
  if (const char* e = getenv("DAB_CHOL_V1")) c->v1 = atoi(e) != 0;
  if (const char* e = getenv("DAB_CHOL_STRIP")) c->strip = atoi(e) != 0;
  if (const char* e = getenv("DAB_CHOL_GROUP")) c->group = std::max(2, atoi(e));
  if (const char* e = getenv("DAB_CHOL_BACK_FLOW")) c->back_flow = atoi(e) != 0;
  if (const char* e = getenv("DAB_CHOL_PREFACTOR")) c->prefactor = atoi(e) != 0;
  if (const char* e = getenv("DAB_CHOL_FUSE_PANEL")) c->fuse_panel = atoi(e) != 0;
  c->nograph = getenv("DAB_CHOL_NOGRAPH") != nullptr;
  if (const char* e = getenv("DAB_CHOL_GRAPH_MIN")) c->graph_min = atoi(e);
  c->serial = getenv("DAB_CHOL_SERIAL") != nullptr;
  // the side stream and the barrier word now, not inside the first solve. (A warm-up graph
  // capture here bought nothing: every instantiation costs ~5 ms, the first one no more.)
  int dev_now = 0;
  (void)hipGetDevice(&dev_now);
  c->device = dev_now;
  if (!(c->side = stream_take(dev_now)) || c->mem.alloc(&c->bar, 1) != 0) {
    chol_destroy(c);
    return nullptr;
  }
  return c;
}
void chol_destroy(CholCtx* c) {
  if (!c) return;
  if (c->exec) (void)hipGraphExecDestroy(c->exec);
  c->mem.clear();
  for (hipEvent_t e : c->ev_panel) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->ev_bulk) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->ev_strip) (void)hipEventDestroy(e);
  stream_give(c->device, c->side);
  delete c;
}

// ---- panel step in one launch --------------------------------------------------------
// Every work-group factors the 64x64 diagonal block itself (blocked by 16: wave 0 factors
// and inverts each 16x16 diagonal block in registers, lane = row, broadcasts by
// v_readlane; the work-group solves the rows below it with that inverse and applies the
// rank-16 update in LDS), then solves its own 64 panel rows P <- P L_kk^-T block column by
// block column with the four 16x16 inverses. Work-group 0 also stores L_kk and the
// inverses (for the back substitution). The redundant factorisations run side by side,
// so the dependent chain per step is one launch instead of potrf -> inverse -> trsm.
constexpr int LS = NB + 1;
constexpr int DS = 17;
// y's "not yet solved" pattern for the back substitution (both 32-bit halves: the double
// 0x7FF47FF47FF47FF4, a signalling NaN, which no arithmetic produces)
constexpr unsigned kYPending32 = 0x7FF47FF4u;
#ifdef DAB_CHOL_PROFILE  // phase timestamps of work-group 0 (scripts/potrf_micro.hip only)
__device__ long long g_prof[16];
#define PROF_MARK(i) \
  if (blockIdx.x == 0 && threadIdx.x == 0) g_prof[i] = wall_clock64();
#else
#define PROF_MARK(i)
#endif
#ifdef DAB_CHOL_STAMPS  // per-work-group phase stamps of the factorisation's launches (A/B builds only)
constexpr int kStampWg = 512, kStampCb = 128;
__device__ unsigned long long g_stamp[3 * kStampCb * kStampWg * 8];  // [kind][block column][wg][phase]
#define CHOL_STAMP(kind, cb, p)                                                                              \
  if (threadIdx.x == 0 && (cb) >= 0 && (cb) < kStampCb && (int)blockIdx.x < kStampWg)                      \
    g_stamp[(((size_t)(kind) * kStampCb + (cb)) * kStampWg + blockIdx.x) * 8 + (p)] = __builtin_amdgcn_s_memrealtime();
#else
#define CHOL_STAMP(kind, cb, p)
#endif

// 1/sqrt(d): v_rsq_f64 and two Newton steps
__device__ __forceinline__ double rsqrt_nr(double d) {
  double y = __builtin_amdgcn_rsq(d);
  y = y * fma(-0.5 * d * y, y, 1.5);
  y = y * fma(-0.5 * d * y, y, 1.5);
  return y;
}


// lane j of each 16-lane row to the whole row as ONE 64-bit DPP move (v_mov_b64_dpp
// row_newbcast: a VGPR broadcast, no SGPR round trip; two 32-bit moves before round 6)
template <int J>
__device__ __forceinline__ double bc64(double v) {
  return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + J, 0xf, 0xf, true);
}
template <int I = 0>
__device__ __forceinline__ double bc64_rt(double v, int j) {  // j a constant after unrolling
  if constexpr (I >= 16) return v;
  else return j == I ? bc64<I>(v) : bc64_rt<I + 1>(v, j);
}

// wave 0: factor L[o:o+16, o:o+16] in place (lane r = row r, the four 16-lane rows of the
// wave redundant), its inverse into D[16][DS] by columns (lane c: column c). Round 6: the
// chain of the dense Cholesky runs this 4 times per 64-block column, twice per panel pair
// on the critical path, and it was instruction bound (1,416 instructions, 3.2 us per call:
// 272 32-bit DPP moves, 140 selects, 124 AGPR spill moves, a finiteness test per pivot).
// Now every broadcast is one v_mov_b64_dpp consumed at once (no AGPR spills), L[r][j] =
// a[j] / sqrt(d) is one multiply for every lane (lane j's a[j] IS d), and the pivots are
// checked once at the end (a pivot d <= 0, NaN or inf makes sum d or sum 1/sqrt(d)
// non-finite). Every value is the same operation on the same operands as before: bitwise
// the same factor and inverse.
typedef __attribute__((address_space(3))) double lds_f64;
__device__ __noinline__ void factor16(double (*Lg)[LS], double (*Dg)[DS], int o, bool& bad) {
  const int lane = threadIdx.x & 63, r = lane & 15;
  // the blocks live in LDS: LDS-typed pointers, so the accesses need no generic-address
  // null checks (the __noinline__ call passes generic pointers)
  lds_f64* Lr = (lds_f64*)(&Lg[o + r][o]);
  lds_f64* Dc = (lds_f64*)(&Dg[0][r]);
  // unconditional (the block's own rows); lane r's entries j > r (the strict upper part,
  // whatever it holds) are only ever used by lane r itself, and nothing reads the upper part
  // of a diagonal 16 x 16 block afterwards (factor64's stages and the panel solves read the
  // blocks below it, the stores of L_kk write zeros there), so it is written back as computed
  double a[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) a[j] = Lr[j];
  // lane c also carries column c of the inverse, x[i] = (delta_ic - sum_{c<=m<i} L[i][m]
  // x[m]) / L[i][i]: its sums take each multiplier L[l][j] from the factorisation's own
  // broadcast of pivot j (x[j] is final once pivot j's 1/L[j][j] is known), so the 120
  // broadcasts serve both and none stays live (a separate inverse loop after the factor
  // shared them by CSE and spilled them to AGPRs)
  const int cc = r;
  double s[16], x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) s[i] = (i == cc) ? 1.0 : 0.0;
  double sd = 0.0, sy = 0.0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const double d = bc64_rt(a[j], j);
    const double y = rsqrt_nr(d);
    sd += d;
    sy += y;
    const double lmj = a[j] * y;  // lane j: d * y = L[j][j]
    a[j] = lmj;
    const double nl = -lmj;
    x[j] = s[j] * y;  // +0 for j < cc: s[j] stays exactly +0 there (every x it saw was +0)
    const double nx = -x[j];
    // lanes r < l update entries above the diagonal that are never read: no mask
#pragma unroll
    for (int l = j + 1; l < 16; ++l) {
      const double b = bc64_rt(lmj, l);  // L[l][j]
      a[l] = fma(b, nl, a[l]);
      s[l] = fma(b, nx, s[l]);
      // the inverse's update here, not deferred: left to itself the scheduler sinks these
      // off-critical-path fmas and keeps the broadcasts b live (spilled to AGPRs)
      asm volatile("" : "+v"(s[l]));
    }
  }
  bad |= !isfinite(sd) || !isfinite(sy);
  if (lane < 16) {  // stores without branches: the strict upper part is written back as read
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      Lr[j] = a[j];
      Dc[j * DS] = x[j];
    }
  }
}

// 16x16 tiles on fp64 MFMA (v_mfma_f64_16x16x4f64; A: lane l holds A[l&15][l>>4], B:
// B[l>>4][l&15], C/D: C[(l>>4) + 4r][l&15]). acc += sign * A B with A(i,k) = As[i0+i][ka+k]
// and B(k,j) = Bt[j0+j][kb+k] (B given transposed, as the row-major factor blocks are).
template <int SA, int SB>
__device__ __forceinline__ void mma_nt(int K, dbl4& acc, const double* As, int i0, int ka, const double* Bt, int j0,
                                       int kb, double sign) {
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int ks = 0; ks < K / 4; ++ks) {
    const double a = sign * As[(i0 + li) * SA + ka + 4 * ks + lk];
    const double b = Bt[(j0 + li) * SB + kb + 4 * ks + lk];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
}
template <int S>
__device__ __forceinline__ dbl4 tile_load(const double* M, int i0, int j0) {
  const int lane = threadIdx.x & 63;
  dbl4 t;
#pragma unroll
  for (int r = 0; r < 4; ++r) t[r] = M[(i0 + (lane >> 4) + 4 * r) * S + j0 + (lane & 15)];
  return t;
}
template <int S>
__device__ __forceinline__ void tile_store(double* M, int i0, int j0, const dbl4& t) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < 4; ++r) M[(i0 + (lane >> 4) + 4 * r) * S + j0 + (lane & 15)] = t[r];
}

// the 64x64 diagonal block (in LDS) -> L in place, D[p] = inverse of its p-th 16x16 block
__device__ __forceinline__ void factor64(double (*L)[LS], double (*D)[16][DS], bool& bad) {
  const int tid = threadIdx.x, w = tid >> 6;
  double* Lf = &L[0][0];
#pragma unroll 1
  for (int p = 0; p < 4; ++p) {
    const int o = 16 * p;
    if (w == 0) factor16(L, D[p], o, bad);
    __syncthreads();
    PROF_MARK(2 + 2 * p);
    if (p == 3) break;
    const int nrc = 3 - p;  // 16-row chunks below the diagonal block
    // block column p below the diagonal: L_R = A_R D_p^T (wave w: chunk w)
    if (w < nrc) {
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
      mma_nt<LS, DS>(16, acc, Lf, o + 16 + 16 * w, o, &D[p][0][0], 0, 0, 1.0);
      __builtin_amdgcn_wave_barrier();
      tile_store<LS>(Lf, o + 16 + 16 * w, o, acc);
    }
    __syncthreads();
    // rank-16 update of the trailing lower tiles (ti >= tj), round robin over waves 0-3
    for (int t = w; w < 4 && t < nrc * (nrc + 1) / 2; t += 4) {
      int ti = 0;
      while ((ti + 1) * (ti + 2) / 2 <= t) ++ti;
      const int tj = t - ti * (ti + 1) / 2;
      const int ri = o + 16 + 16 * ti, rj = o + 16 + 16 * tj;
      dbl4 acc = tile_load<LS>(Lf, ri, rj);
      mma_nt<LS, LS>(16, acc, Lf, ri, o, Lf, rj, o, -1.0);
      tile_store<LS>(Lf, ri, rj, acc);
    }
    __syncthreads();
    PROF_MARK(3 + 2 * p);
  }
}

// One wave's 16 panel rows P (LDS, stride LS) <- P L_kk^-T, block column by block column:
// X_q = (P_q - sum_{r<q} X_r L_{q,r}^T) D_q^T. Right-looking (round 6): as soon as X_q is
// known its term goes into every later block's accumulator, so the dependent chain is
// X_q -> the next block's last 4 MFMAs -> X_{q+1} (28 MFMAs deep instead of 40; the other
// blocks' updates overlap it). Each block's accumulator still takes the terms r = 0, 1, ...
// in order, the same MFMAs on the same operands as the left-looking form: bitwise the same.
__device__ __forceinline__ void panel_rows_solve(double* Pf, const double* Lf, const double (*D)[16][DS], int w) {
  dbl4 acc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = tile_load<LS>(Pf, 16 * w, 16 * q);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    __builtin_amdgcn_wave_barrier();
    tile_store<LS>(Pf, 16 * w, 16 * q, acc[q]);
    __builtin_amdgcn_wave_barrier();
    dbl4 x = {0.0, 0.0, 0.0, 0.0};
    mma_nt<LS, DS>(16, x, Pf, 16 * w, 16 * q, &D[q][0][0], 0, 0, 1.0);
    __builtin_amdgcn_wave_barrier();
    tile_store<LS>(Pf, 16 * w, 16 * q, x);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int qq = q + 1; qq < 4; ++qq) mma_nt<LS, LS>(16, acc[qq], Pf, 16 * w, 16 * q, Lf, 16 * qq, 16 * q, -1.0);
  }
}

// panel rows [r0, r1) (64 per work-group): P <- P L_kk^-T ; work-group 0 stores D and L_kk
// to the block scratch
// pre: the diagonal block was factored by the column update in front (k_syrk_mfma with
// fblk), so L_kk and the inverses are read from the block scratch instead
// yinit / pinit (the factorisation's first panel): the launch also sets y[0, ny) to the
// back substitution's pending pattern and zeroes pinit[0, np) (the fused steps' flags), so
// that neither is a fill on the chain
__global__ __launch_bounds__(kThreads) void k_panel(double* __restrict__ A, int lda, int k, int kb, int r0,
                                                    int r1, double* __restrict__ blk, int* __restrict__ flag,
                                                    int pre, double* __restrict__ yinit = nullptr, int ny = 0,
                                                    unsigned* __restrict__ pinit = nullptr, int np = 0) {
  __shared__ double L[NB][LS];
  __shared__ double P[NB][LS];
  __shared__ double D[4][16][DS];
  // the panel chain is the critical path: its waves win the issue arbitration against the
  // bulk update's waves on shared CUs
  __builtin_amdgcn_s_setprio(3);
  const int tid = threadIdx.x, w = tid >> 6;
  for (int i = blockIdx.x * kThreads + tid; i < ny; i += gridDim.x * kThreads)
    yinit[i] = __longlong_as_double((long long)(((unsigned long long)kYPending32 << 32) | kYPending32));
  for (int i = blockIdx.x * kThreads + tid; i < np; i += gridDim.x * kThreads) pinit[i] = 0u;
  const int row0 = r0 + NB * blockIdx.x;
  if (pre) {
    if (row0 >= r1) return;
#pragma unroll
    for (int q = 0; q < NB * NB / kThreads; ++q) {
      const int idx = tid + q * kThreads, i = idx >> 6, j = idx & 63;
      L[i][j] = blk[1024 + idx];
      P[i][j] = (row0 + i < r1 && j < kb) ? A[(size_t)(row0 + i) * lda + k + j] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + q * kThreads;
      D[idx >> 8][(idx >> 4) & 15][idx & 15] = blk[idx];
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < NB * NB / kThreads; ++q) {
    if (pre) break;
    const int idx = tid + q * kThreads, i = idx >> 6, j = idx & 63;
    double v = (i == j) ? 1.0 : 0.0;
    if (i < kb && j <= i) v = A[(size_t)(k + i) * lda + k + j];
    L[i][j] = v;
    P[i][j] = (row0 + i < r1 && j < kb) ? A[(size_t)(row0 + i) * lda + k + j] : 0.0;
  }
  PROF_MARK(0);
  if (!pre) __syncthreads();
  PROF_MARK(1);
  bool bad = false;
  if (!pre) factor64(L, D, bad);
  if (blockIdx.x == 0 && !pre) {
    // L_kk goes to the scratch, not back into A: the other work-groups of this launch
    // may not have read the original diagonal block yet
    if (tid == 0 && bad) atomicOr(flag, 1);
#pragma unroll
    for (int q = 0; q < NB * NB / kThreads; ++q) {
      const int idx = tid + q * kThreads, i = idx >> 6, j = idx & 63;
      blk[1024 + idx] = (j <= i) ? L[i][j] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + q * kThreads;  // [4][16][16]
      blk[idx] = D[idx >> 8][(idx >> 4) & 15][idx & 15];
    }
  }
  if (row0 >= r1) return;
  // wave w solves rows [16w, 16w+16) of P (no barriers: the rows are its own)
  panel_rows_solve(&P[0][0], &L[0][0], D, w);
  __syncthreads();
  PROF_MARK(10);
#pragma unroll
  for (int q = 0; q < NB * NB / kThreads; ++q) {
    const int idx = tid + q * kThreads, i = idx >> 6, j = idx & 63;
    if (row0 + i < r1 && j < kb) A[(size_t)(row0 + i) * lda + k + j] = P[i][j];
  }
}

// col_only: just the first tile column of the trailing matrix (tile (t, 0)), the block
// column the next panel step factors; otherwise the whole lower triangle of tiles.
// ntiles: tiles of the launch; the grid may be smaller (a persistent bulk update that leaves
// every CU room for the panel chain's work-groups), each work-group loops over its tiles.
// The update has rank kk: panel columns [k, k + kk) in chunks of NB (kk = kb of one panel,
// or two panels' 128 for the column after a panel pair).
// fblk (col_only): the work-group of the diagonal tile then factors it (factor64, the first
// kb_next rows; identity below) and stores L_kk and the 16x16 inverses there, so that the
// next panel (k_panel pre) reads them instead of every work-group factoring the block.
// ready (with fblk): the panel step is fused in as well — the diagonal work-group publishes
// L_kk and the inverses (agent-scope stores, then ready = 1) and every other work-group
// keeps its updated tile, which is its 64 panel rows, waits for ready (bounded: flag |= 2)
// and solves the rows P <- P L_kk^-T (as k_panel), so the chain loses a launch per block.
// FACTOR: the fblk / ready paths are compiled in (their factor16 calls hold the kernel at 373
// registers per lane, one wave per SIMD); the plain update (strips, the per-step schedule) is
// the FACTOR = false instance.
template <bool FACTOR>
__global__ __launch_bounds__(kThreads) void k_syrk_mfma(double* __restrict__ A, int lda, int r0, int m, int k0,
                                                        int kk, int col_only, int ntiles,
                                                        double* __restrict__ fblk = nullptr, int kb_next = 0,
                                                        int* __restrict__ flag = nullptr,
                                                        unsigned* __restrict__ ready = nullptr) {
  __shared__ double Pa[NB * LDP];
  __shared__ double Pb[NB * LDP];
  __shared__ double Dsh[4][16][DS];
  __shared__ int abort_s;
  if (col_only) __builtin_amdgcn_s_setprio(3);  // on the panel chain
  [[maybe_unused]] const int skind = fblk ? 0 : 1, scb = col_only ? r0 / NB : -1;
  CHOL_STAMP(skind, scb, 0);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
  if (t != (int)blockIdx.x) __syncthreads();  // the previous tile's LDS reads are done
  int bi = t, bj = 0;
  if (!col_only) {
    bi = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((bi + 1) * (bi + 2) / 2 <= t) ++bi;
    while (bi * (bi + 1) / 2 > t) --bi;
    bj = t - bi * (bi + 1) / 2;
  }
  const int tid = threadIdx.x;
  const bool diag = bi == bj;
  const int w = tid >> 6, lane = tid & 63;
  const int wr = w >> 1, wc = w & 1;  // 32x32 quadrant of the tile
  const bool skip = diag && wr < wc;  // strictly upper quadrant of a diagonal tile
  const int li = lane & 15, lk = lane >> 4;
  // the accumulators start as the C tile (issued first, so its HBM latency overlaps the
  // panel staging); the MFMAs then add -P_i P_j^T
  dbl4 acc[2][2];
#pragma unroll
  for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
    for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int row = bi * NB + wr * 32 + a2 * 16 + lk + 4 * reg;
        const int col = bj * NB + wc * 32 + b2 * 16 + li;
        // clamped, unconditional: an element outside the matrix (or in a skipped quadrant)
        // is never stored, and no stored element depends on it
        acc[a2][b2][reg] = A[(size_t)(r0 + min(row, m - 1)) * lda + r0 + min(col, m - 1)];
      }
  for (int k = k0; k < k0 + kk; k += NB) {
  const int kb = min(NB, k0 + kk - k);
  if (k != k0) __syncthreads();  // the previous chunk's LDS reads are done
  // coalesced tile loads: 8 rows per pass, 32 double2 per row. Every load unconditional
  // (row and column clamped into the matrix; a row past m only feeds outputs that are never
  // stored), the columns past kb zeroed by a 0/1 factor: a select or a branch here made
  // hipcc wait for each load before the next (one L2 round trip per row pass)
  const int c2 = tid & 31;
  const int ka = k + min(2 * c2, kb - 1), kb1 = k + min(2 * c2 + 1, kb - 1);
  const double f0 = 2 * c2 < kb ? 1.0 : 0.0, f1 = 2 * c2 + 1 < kb ? 1.0 : 0.0;
  double2 va[NB / 8], vb[NB / 8];
#pragma unroll
  for (int q = 0; q < NB / 8; ++q) {
    const int rr = (tid >> 5) + 8 * q;
    const double* sa = A + (size_t)(r0 + min(bi * NB + rr, m - 1)) * lda;
    va[q] = make_double2(sa[ka], sa[kb1]);
    if (!diag) {
      const double* sb = A + (size_t)(r0 + min(bj * NB + rr, m - 1)) * lda;
      vb[q] = make_double2(sb[ka], sb[kb1]);
    }
  }
#pragma unroll
  for (int q = 0; q < NB / 8; ++q) {
    const int rr = (tid >> 5) + 8 * q;
    *reinterpret_cast<double2*>(&Pa[rr * LDP + 2 * c2]) = make_double2(va[q].x * f0, va[q].y * f1);
    if (!diag) *reinterpret_cast<double2*>(&Pb[rr * LDP + 2 * c2]) = make_double2(vb[q].x * f0, vb[q].y * f1);
  }
  __syncthreads();
  if (k == k0 && t == (int)blockIdx.x) CHOL_STAMP(skind, scb, 1);
  const double* PB = diag ? Pa : Pb;
  if (skip) continue;
#pragma unroll 4
  for (int ks = 0; ks < NB / 4; ++ks) {
    double fa[2], fb[2];
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2) fa[a2] = -Pa[(wr * 32 + a2 * 16 + li) * LDP + ks * 4 + lk];
#pragma unroll
    for (int b2 = 0; b2 < 2; ++b2) fb[b2] = PB[(wc * 32 + b2 * 16 + li) * LDP + ks * 4 + lk];
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
      for (int b2 = 0; b2 < 2; ++b2)
        acc[a2][b2] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[a2], fb[b2], acc[a2][b2], 0, 0, 0);
  }
  }
  // D layout (f64 16x16x4): col = lane & 15, row = (lane >> 4) + 4 * reg
  if (t == (int)blockIdx.x) CHOL_STAMP(skind, scb, 2);
#pragma unroll
  for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
    for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int row = bi * NB + wr * 32 + a2 * 16 + lk + 4 * reg;
        const int col = bj * NB + wc * 32 + b2 * 16 + li;
        if (!skip && row < m && col < m) A[(size_t)(r0 + row) * lda + r0 + col] = acc[a2][b2][reg];
      }
  if (t == (int)blockIdx.x) CHOL_STAMP(skind, scb, 3);
  if (FACTOR && fblk && col_only && bi == 0) {
    // Pb is free on a diagonal tile: it holds L [NB][LS]
    double (*L)[LS] = reinterpret_cast<double (*)[LS]>(Pb);
    double (*D)[16][DS] = Dsh;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NB * NB / kThreads; ++q) {
      const int idx = tid + q * kThreads, i = idx >> 6, j = idx & 63;
      L[i][j] = (i == j) ? 1.0 : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
      for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int i = wr * 32 + a2 * 16 + lk + 4 * reg, j = wc * 32 + b2 * 16 + li;
          if (!skip && i < kb_next && j <= i) L[i][j] = acc[a2][b2][reg];
        }
    __syncthreads();
    bool bad = false;
    factor64(L, D, bad);
    if (tid == 0 && bad) atomicOr(flag, 1);
#pragma unroll
    for (int q = 0; q < NB * NB / kThreads; ++q) {
      const int idx = tid + q * kThreads, i = idx >> 6, j = idx & 63;
      __hip_atomic_store(fblk + 1024 + idx, (j <= i) ? L[i][j] : 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + q * kThreads;  // [4][16][16]
      __hip_atomic_store(fblk + idx, D[idx >> 8][(idx >> 4) & 15][idx & 15], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    if (ready) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(ready, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    CHOL_STAMP(skind, scb, 4);
  } else if (FACTOR && ready && col_only) {
    // the fused panel step on this tile's rows
    double (*P)[LS] = reinterpret_cast<double (*)[LS]>(Pb);
    double (*L)[LS] = reinterpret_cast<double (*)[LS]>(Pa);
    __syncthreads();  // the MFMA loop's LDS reads are done
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
      for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int i = wr * 32 + a2 * 16 + lk + 4 * reg, j = wc * 32 + b2 * 16 + li;
          P[i][j] = j < kb_next ? acc[a2][b2][reg] : 0.0;
        }
    if (tid == 0) {
      abort_s = 0;
      int spins = 0;
      while (__hip_atomic_load(ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1 << 22)) {
          abort_s = 1;
          atomicOr(flag, 2);
          break;
        }
      }
    }
    __syncthreads();
    if (abort_s) return;
    CHOL_STAMP(skind, scb, 4);
#pragma unroll
    for (int q = 0; q < NB * NB / kThreads; ++q) {
      const int idx = tid + q * kThreads, i = idx >> 6, j = idx & 63;
      L[i][j] = __hip_atomic_load(fblk + 1024 + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + q * kThreads;
      Dsh[idx >> 8][(idx >> 4) & 15][idx & 15] = __hip_atomic_load(fblk + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    panel_rows_solve(&P[0][0], &L[0][0], Dsh, w);  // wave w: rows [16 w, 16 w + 16), as k_panel
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NB * NB / kThreads; ++q) {
      const int idx = tid + q * kThreads, i = idx >> 6, j = idx & 63;
      const int row = bi * NB + i;
      if (row < m && j < kb_next) A[(size_t)(r0 + row) * lda + r0 + j] = P[i][j];
    }
  }
  }
  CHOL_STAMP(skind, scb, 5);
}

// back substitution step for block [k, k+kb): y_k = L_kk^-T z_k by 16-blocks with the
// stored inverses D_q (y_q = D_q^T (z_q - sum_{r>q} L_rq^T y_r)), then
// z[0:k] -= L[k:k+kb, 0:k]^T y_k
__global__ __launch_bounds__(kThreads) void k_trsv_back(const double* __restrict__ A, int lda, int k, int kb,
                                                        const double* __restrict__ blk,
                                                        double* __restrict__ z, double* __restrict__ y) {
  __shared__ double Lk[NB][LS];
  __shared__ double Dq[4][16][DS];
  __shared__ double yy[NB];
  __shared__ double tt[16];
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < NB * NB / kThreads; ++q) {
    const int idx = tid + q * kThreads, i = idx >> 6, j = idx & 63;
    Lk[i][j] = blk[1024 + idx];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int idx = tid + q * kThreads;
    Dq[idx >> 8][(idx >> 4) & 15][idx & 15] = blk[idx];
  }
  if (tid < NB) yy[tid] = tid < kb ? z[k + tid] : 0.0;
  __syncthreads();
  if (tid < 64) {  // one wave, lanes 0..15 carry the 16-vectors
    const int c = tid & 15;
#pragma unroll
    for (int q = 3; q >= 0; --q) {
      double t = yy[16 * q + c];
#pragma unroll
      for (int r = q + 1; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 16; ++i) t = fma(-Lk[16 * r + i][16 * q + c], yy[16 * r + i], t);
      if (tid < 16) tt[c] = t;
      __builtin_amdgcn_wave_barrier();
      double s = 0.0;
#pragma unroll
      for (int m = 0; m < 16; ++m)
        if (m >= c) s = fma(Dq[q][m][c], tt[m], s);
      __builtin_amdgcn_wave_barrier();
      if (tid < 16) yy[16 * q + c] = s;
      __builtin_amdgcn_wave_barrier();
    }
  }
  __syncthreads();
  if (blockIdx.x == 0 && tid < kb) y[k + tid] = yy[tid];
  // 64 columns per workgroup, 4 lanes per column (16 rows of the block each)
  const int i = blockIdx.x * (kThreads / 4) + (tid & 63);
  const int part = tid >> 6;
  double s = 0.0;
  if (i < k) {
#pragma unroll
    for (int q = 0; q < NB / 4; ++q) {
      const int mm = part * (NB / 4) + q;
      if (mm < kb) s += A[(size_t)(k + mm) * lda + i] * yy[mm];
    }
  }
  __shared__ double red[4][64];
  red[part][tid & 63] = s;
  __syncthreads();
  if (part == 0 && i < k) z[i] -= ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
}


// Bulk trailing update of a panel PAIR on 128 x 128 super-tiles (rank kk <= 128: the two
// 64-wide panels of the pair, so the trailing matrix is read and written once per two
// panel steps): C(i, j) -= sum_{q in [k0, k0 + kk)} A(i, q) A(j, q) for c0 <= j <= i <
// c0 + m. Persistent: work-group g walks the lower super-tiles t = g, g + grid, ...; each
// super-tile as two 64 x 128 row halves in sequence (units u = 2t + h). Per half the product
// streams through LDS in 16-wide K chunks, double-buffered (the next chunk's global loads in
// flight during the current chunk's MFMAs); wave w owns the 32 x 32 block (w & 1, w >> 1):
// 2 x 2 tiles of v_mfma_f64_16x16x4f64, 16 accumulators per lane. The NEXT unit's C is
// loaded into registers during the current unit's last CP chunks (after their chunk loads:
// vmcnt counts in order), so the trailing matrix's HBM traffic overlaps the MFMAs instead of
// stalling every unit's start (round 5, scripts/syrk_big_probe.hip: 126 -> 118 us at m =
// 5739, 55.5 -> 51-52 us at m = 3939; the whole-tile form's C load and store were serial
// with its MFMAs). Every element is C + the same MFMA sequence in k as before: bitwise the
// same factor. A diagonal super-tile skips its strictly upper 64 x 64 quadrant. All LDS is
// one __shared__ array (a second one can make hipcc drain vmcnt before every ds_read).
constexpr int TB = 128;  // super-tile
constexpr int kBigThreads = 512;
template <int KC, int CP>  // K chunk, chunks of the C prefetch window
__global__ __launch_bounds__(kBigThreads, 4) void k_syrk_big(double* __restrict__ A, int lda, int c0, int m, int k0,
                                                        int kk, int ntiles) {
  constexpr int LKC = KC + 2;
  constexpr int PA = KC / 8;  // A (the half's 64 rows): 8 loader threads per row
  constexpr int PB = KC / 4;  // B (the tile's 128 columns): 4 loader threads per row
  constexpr int SA = 64 * LKC, SS = SA + TB * LKC;
  __shared__ double sm[2 * SS];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, li = lane & 15, lk = lane >> 4;
  const int wrow = 32 * (w & 1), wcol = 32 * (w >> 1);
  const int ar = tid >> 3, ah = (tid & 7) * PA, br = tid >> 2, bh = (tid & 3) * PB;
  const int nch = kk / KC, nunits = 2 * ntiles, ustep = 2 * (int)gridDim.x;
  auto coords = [&](int t, int& bi, int& bj) {
    bi = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((bi + 1) * (bi + 2) / 2 <= t) ++bi;
    while (bi * (bi + 1) / 2 > t) --bi;
    bj = t - bi * (bi + 1) / 2;
  };
  auto cload = [&](int u, dbl4(&cv)[2][2]) {
    int bi, bj;
    coords(u >> 1, bi, bj);
    const int r0 = bi * TB + 64 * (u & 1) + wrow, q0 = bj * TB + wcol;
#pragma unroll
    for (int tr = 0; tr < 2; ++tr)
#pragma unroll
      for (int tc = 0; tc < 2; ++tc)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int row = r0 + 16 * tr + lk + 4 * reg, col = q0 + 16 * tc + li;
          // clamped address, no select: an element outside the matrix is never stored, and
          // no element inside depends on it (a select here becomes a branch + wait per load)
          cv[tr][tc][reg] = A[(size_t)(c0 + min(row, m - 1)) * lda + c0 + min(col, m - 1)];
        }
  };
  CHOL_STAMP(2, c0 / NB, 0);
  dbl4 acc[2][2], nxt[2][2];
  int u = 2 * (int)blockIdx.x;
  if (u < nunits) cload(u, acc);
  while (u < nunits) {
    const int h = u & 1;
    int bi, bj;
    coords(u >> 1, bi, bj);
    const bool skip = bi == bj && (w >> 2) > h;  // a strictly upper 64 x 64 quadrant
    const int ri0 = bi * TB + 64 * h, rj0 = bj * TB;
    double ra[PA], rb[PB];
    const double* srca = A + (size_t)(c0 + min(ri0 + ar, m - 1)) * lda + k0 + ah;
    const double* srcb = A + (size_t)(c0 + min(rj0 + br, m - 1)) * lda + k0 + bh;
    auto gload = [&](int ch) {
#pragma unroll
      for (int q = 0; q < PA; ++q) ra[q] = srca[ch * KC + q];
#pragma unroll
      for (int q = 0; q < PB; ++q) rb[q] = srcb[ch * KC + q];
    };
    auto sstore = [&](int st) {
      double* a = sm + (size_t)st * SS + ar * LKC + ah;
#pragma unroll
      for (int q = 0; q < PA; q += 2) *reinterpret_cast<double2*>(a + q) = make_double2(ra[q], ra[q + 1]);
      double* b = sm + (size_t)st * SS + SA + br * LKC + bh;
#pragma unroll
      for (int q = 0; q < PB; q += 2) *reinterpret_cast<double2*>(b + q) = make_double2(rb[q], rb[q + 1]);
    };
    const int un = h == 0 ? u + 1 : u - 1 + ustep;
    const int unc = min(un, nunits - 1);  // clamped: the prefetch is unconditional
    gload(0);
    __syncthreads();
    sstore(0);
    __syncthreads();
    const int cpre = nch >= CP ? nch - CP : 0;
    for (int ch = 0; ch < nch; ++ch) {
      const int st = ch & 1;
      if (ch + 1 < nch) gload(ch + 1);
      if (ch == cpre) cload(unc, nxt);  // after the half's last chunk load (in-order vmcnt)
      if (!skip) {
        const double* As = sm + (size_t)st * SS;
        const double* Bs = As + SA;
#pragma unroll
        for (int ks = 0; ks < KC / 4; ++ks) {
          double fa[2], fb[2];
#pragma unroll
          for (int tr = 0; tr < 2; ++tr) fa[tr] = -As[(wrow + 16 * tr + li) * LKC + 4 * ks + lk];
#pragma unroll
          for (int tc = 0; tc < 2; ++tc) fb[tc] = Bs[(wcol + 16 * tc + li) * LKC + 4 * ks + lk];
#pragma unroll
          for (int tr = 0; tr < 2; ++tr)
#pragma unroll
            for (int tc = 0; tc < 2; ++tc)
              acc[tr][tc] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[tr], fb[tc], acc[tr][tc], 0, 0, 0);
        }
      }
      if (ch + 1 < nch) sstore(st ^ 1);
      __syncthreads();
    }
    if (!skip) {
#pragma unroll
      for (int tr = 0; tr < 2; ++tr)
#pragma unroll
        for (int tc = 0; tc < 2; ++tc)
#pragma unroll
          for (int reg = 0; reg < 4; ++reg) {
            const int row = ri0 + wrow + 16 * tr + lk + 4 * reg, col = rj0 + wcol + 16 * tc + li;
            if (row < m && col < m) A[(size_t)(c0 + row) * lda + c0 + col] = acc[tr][tc][reg];
          }
    }
#pragma unroll
    for (int tr = 0; tr < 2; ++tr)
#pragma unroll
      for (int tc = 0; tc < 2; ++tc) acc[tr][tc] = nxt[tr][tc];
    u = un;
  }
  CHOL_STAMP(2, c0 / NB, 5);
}


// Back substitution L^T y = z in ONE launch (instead of one per block): grid G <= CUs,
// every work-group resident. Per block b, last first, every work-group computes y_b =
// L_bb^-T z_b from the stored 16x16 inverses (redundantly: no hand-off needed for it),
// work-group 0 writes y_b, and each work-group updates its 64-column shares of z[0:k_b]
// with L[k_b : k_b + kb, shares]^T y_b; then a grid barrier (the counter form of the
// agent-scope release/acquire hand-off; bounded spin: on timeout flag |= 2 and the kernel
// ends instead of hanging).
__global__ __launch_bounds__(kThreads) void k_trsv_back_all(const double* __restrict__ A, int lda, int n, int nblk,
                                                            const double* __restrict__ blk, double* __restrict__ z,
                                                            double* __restrict__ y, unsigned* __restrict__ bar,
                                                            int* __restrict__ flag) {
  __shared__ double Lk[NB][LS];
  __shared__ double Dq[4][16][DS];
  __shared__ double yy[NB];
  __shared__ double tt[16];
  __shared__ double red[4][64];
  __shared__ int abort_s;
  const int tid = threadIdx.x, G = gridDim.x;
  if (tid == 0) abort_s = 0;
  for (int b = nblk - 1; b >= 0; --b) {
    const int k = b * NB, kb = min(NB, n - k);
    const double* bk = blk + (size_t)b * kBlk;
#pragma unroll
    for (int q = 0; q < NB * NB / kThreads; ++q) {
      const int idx = tid + q * kThreads, i = idx >> 6, j = idx & 63;
      Lk[i][j] = bk[1024 + idx];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + q * kThreads;
      Dq[idx >> 8][(idx >> 4) & 15][idx & 15] = bk[idx];
    }
    // z_b: written by its owner with agent-scope (L2-bypassing) stores, read likewise
    if (tid < NB) yy[tid] = tid < kb ? __hip_atomic_load(z + k + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
    __syncthreads();
    // y_b by 16-blocks, q = 3..0, with all 256 threads (c = tid & 15, part = tid >> 4):
    // t_c = z_c - sum_{j >= 16 (q+1)} L[j][16 q + c] y_j (terms j = 16 (q+1) + part + 16 u),
    // then y_{16 q + c} = sum_{mm >= c} D_q[mm][c] t_mm (term mm = part); both sums in a fixed
    // order through LDS
    {
      const int c = tid & 15, part = tid >> 4;
#pragma unroll
      for (int q = 3; q >= 0; --q) {
        double acc = 0.0;
        for (int j = 16 * (q + 1) + part; j < NB; j += 16) acc = fma(-Lk[j][16 * q + c], yy[j], acc);
        red[part >> 2][(part & 3) * 16 + c] = acc;
        __syncthreads();
        if (tid < 16) {
          double t = yy[16 * q + c];
#pragma unroll
          for (int p2 = 0; p2 < 16; ++p2) t += red[p2 >> 2][(p2 & 3) * 16 + c];
          tt[c] = t;
        }
        __syncthreads();
        red[part >> 2][(part & 3) * 16 + c] = part >= c ? Dq[q][part][c] * tt[part] : 0.0;
        __syncthreads();
        if (tid < 16) {
          double sacc = 0.0;
#pragma unroll
          for (int p2 = 0; p2 < 16; ++p2) sacc += red[p2 >> 2][(p2 & 3) * 16 + c];
          yy[16 * q + c] = sacc;
        }
        __syncthreads();
      }
    }
    if (blockIdx.x == 0 && tid < kb) y[k + tid] = yy[tid];
    if (b == 0) break;
    // z[i] -= sum_mm L[k + mm][i] y[mm] for this work-group's 64-column shares of [0, k)
    const int part = tid >> 6;
    for (int i0 = blockIdx.x * 64; i0 < k; i0 += 64 * G) {
      const int i = i0 + (tid & 63);
      double sacc = 0.0;
      if (i < k) {
#pragma unroll
        for (int q = 0; q < NB / 4; ++q) {
          const int mm = part * (NB / 4) + q;
          if (mm < kb) sacc += A[(size_t)(k + mm) * lda + i] * yy[mm];
        }
      }
      red[part][tid & 63] = sacc;
      __syncthreads();
      if (part == 0 && i < k) {
        // z[i] has one writer (this work-group, every step): the current value is its own
        const double zi = __hip_atomic_load(z + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(z + i, zi - (((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
    }
    // grid barrier: every wave's (agent-scope) z stores complete before the ticket; a
    // bounded relaxed poll. No cache-wide release/acquire: z moves by agent-scope accesses
    // only, and L_bb, D_b, A stay cached.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)G * (unsigned)(nblk - b);
      int spins = 0;
      while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1 << 22)) {
          abort_s = 1;
          atomicOr(flag, 2);
          break;
        }
      }
    }
    __syncthreads();
    if (abort_s) return;
  }
}

// Back substitution L^T y = z as a dataflow over the blocks (no grid barrier): work-group
// w owns the blocks s = w, w + G, ... and keeps their z_s in LDS. For b = last .. 1 it
// waits for y_b (published by b's owner: agent-scope stores, then ready[b]), subtracts
// L_bs^T y_b from each owned z_s with s < b, and when it owns b - 1 — whose z is then
// final — solves y_{b-1} = L^-T z from the stored 16x16 inverses and publishes it. Only
// that owner is on the critical path per block; everyone else consumes y_b in parallel.
// The A block of the critical owned column is loaded before the wait. Waits are bounded
// (flag |= 2 and the work-group ends). Every work-group must be resident (G <= CUs).
// Round 6: y itself is the flag. It is filled with a signalling-NaN pattern before the
// launch (no arithmetic result has that bit pattern: computed NaNs are quiet), the owner
// stores y_b with agent-scope stores and nothing else, and a consumer polls y_b's 64 values
// until none is the pattern — one memory round trip per block on the chain instead of two
// (flag, then values) plus the owner's wait for its stores before the flag.
constexpr int kMaxOwned = 4;
__device__ __forceinline__ bool y_pending(double v) {
  return __double_as_longlong(v) == (long long)(((unsigned long long)kYPending32 << 32) | kYPending32);
}
__global__ __launch_bounds__(kThreads) void k_trsv_back_flow(const double* __restrict__ A, int lda, int n, int nblk,
                                                             const double* __restrict__ blk,
                                                             const double* __restrict__ z, double* __restrict__ y,
                                                             int* __restrict__ flag) {
  __shared__ double Lk[NB][LS];
  __shared__ double Li[NB][LS];  // L_bb^-1 of the next owned block (built off the critical path)
  __shared__ double Dq[4][16][DS];
  __shared__ double zs[kMaxOwned][NB];
  __shared__ double yy[NB];
  __shared__ double red[4][64];
  __shared__ int abort_s;
  const int tid = threadIdx.x, G = gridDim.x, w = blockIdx.x;
  const int nown = w < nblk ? (nblk - 1 - w) / G + 1 : 0;  // owned: s_j = w + G j
  if (tid == 0) abort_s = 0;
  for (int j = 0; j < nown; ++j) {
    const int k = (w + G * j) * NB, kb = min(NB, n - k);
    if (tid < NB) zs[j][tid] = tid < kb ? z[k + tid] : 0.0;
  }
  // L_bb^-1 of block sb from L_bb and the inverses D_q of its 16x16 diagonal blocks, by
  // 16-block rows: Li_qq = D_q, Li_pq = -D_p sum_{q <= r < p} L_pr Li_rq (ends with a barrier)
  auto load_tabs = [&](int sb) {
    const double* bk = blk + (size_t)sb * kBlk;
#pragma unroll
    for (int q = 0; q < NB * NB / kThreads; ++q) {
      const int idx = tid + q * kThreads, i = idx >> 6, jj = idx & 63;
      Lk[i][jj] = bk[1024 + idx];
      Li[i][jj] = 0.0;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + q * kThreads;
      Dq[idx >> 8][(idx >> 4) & 15][idx & 15] = bk[idx];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + q * kThreads, qq = idx >> 8, i = (idx >> 4) & 15, jj = idx & 15;
      Li[16 * qq + i][16 * qq + jj] = i >= jj ? Dq[qq][i][jj] : 0.0;  // lower part only
    }
    __syncthreads();
    for (int p = 1; p < 4; ++p) {
      // T = sum_r L_pr Li_rq for the p blocks q < p (16 x 16 each): 256 threads over (q, i, j)
      double T[3];
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int idx = tid + u * kThreads, q = idx >> 8, i = (idx >> 4) & 15, jj = idx & 15;
        double t = 0.0;
        if (q < p)
          for (int m = 16 * q; m < 16 * p; ++m) t = fma(Lk[16 * p + i][m], Li[m][16 * q + jj], t);
        T[u] = t;
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 3; ++u) {  // park T in the (still zero) block Li_pq
        const int idx = tid + u * kThreads, q = idx >> 8, i = (idx >> 4) & 15, jj = idx & 15;
        if (q < p) Li[16 * p + i][16 * q + jj] = T[u];
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int idx = tid + u * kThreads, q = idx >> 8, i = (idx >> 4) & 15, jj = idx & 15;
        double t = 0.0;
        if (q < p)
          for (int m = 0; m <= i; ++m) t = fma(Dq[p][i][m], Li[16 * p + m][16 * q + jj], t);
        T[u] = -t;
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int idx = tid + u * kThreads, q = idx >> 8, i = (idx >> 4) & 15, jj = idx & 15;
        if (q < p) Li[16 * p + i][16 * q + jj] = T[u];
      }
      __syncthreads();
    }
  };
  // y_sb = (L_bb^-1)^T zs[j] (4 lanes per row, fixed-order sum), then publish
  auto solve_publish = [&](int j) {
    const int sb = w + G * j, k = sb * NB, kb = min(NB, n - k);
    {
      const int i = tid & 63, part = tid >> 6;
      double acc = 0.0;
      for (int m = i + part; m < NB; m += 4) acc = fma(Li[m][i], zs[j][m], acc);
      red[part][i] = acc;
    }
    __syncthreads();
    if (tid < NB) yy[tid] = ((red[0][tid] + red[1][tid]) + red[2][tid]) + red[3][tid];
    if (tid < kb) __hip_atomic_store(y + k + tid, yy[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
  };
  if (nown == 0) return;
  int jn = nown - 1;  // the next owned block to solve (largest s first)
  load_tabs(w + G * jn);
  if (w + G * jn == nblk - 1) {
    solve_publish(jn);
    --jn;
    if (jn >= 0) load_tabs(w + G * jn);
  }
  const int i = tid & 63, part = tid >> 6;
  for (int b = nblk - 1; b >= 1 && jn >= 0; --b) {
    // owned blocks below b: j = 0 .. jmax (s_j < b)
    const int jmax = min(nown - 1, (b - 1 - w) / G);
    if (b - 1 < w) break;
    const int kbk = b * NB, kbb = min(NB, n - kbk);
    // the critical owned column (the largest s < b) is loaded before the wait
    double pa[NB / 4];
    {
      const int col = (w + G * jmax) * NB + i;
#pragma unroll
      for (int q = 0; q < NB / 4; ++q) {
        const int mm = part * (NB / 4) + q;
        pa[q] = (mm < kbb && col < n) ? A[(size_t)(kbk + mm) * lda + col] : 0.0;
      }
    }
    if (tid < NB) {  // wave 0 polls y_b until every value has landed
      double v = 0.0;
      int spins = 0;
      for (;;) {
        v = tid < kbb ? __hip_atomic_load(y + kbk + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
        if (!__any(y_pending(v))) break;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1 << 22)) {
          if (tid == 0) {
            abort_s = 1;
            atomicOr(flag, 2);
          }
          break;
        }
      }
      yy[tid] = v;
    }
    __syncthreads();
    if (abort_s) return;
    for (int j = jmax; j >= 0; --j) {
      const int col = (w + G * j) * NB + i;
      double sacc = 0.0;
#pragma unroll
      for (int q = 0; q < NB / 4; ++q) {
        const int mm = part * (NB / 4) + q;
        const double a = j == jmax ? pa[q] : ((mm < kbb && col < n) ? A[(size_t)(kbk + mm) * lda + col] : 0.0);
        sacc = fma(a, yy[mm], sacc);
      }
      red[part][i] = sacc;
      __syncthreads();
      if (part == 0) zs[j][i] -= ((red[0][i] + red[1][i]) + red[2][i]) + red[3][i];
      __syncthreads();
    }
    if (jmax == jn && w + G * jn == b - 1) {  // z_{b-1} is final
      solve_publish(jn);
      --jn;
      if (jn >= 0) load_tabs(w + G * jn);
    }
  }
}

static void enqueue_factor_solve(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y,
                                 int* d_flag);

static int chol_build(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y, int* d_flag, bool launch);
#ifdef DAB_CHOL_STAMPS
// the stamps of one factorisation (the 4th of the process), per launch: for each phase the
// median and max over work-groups, in us from the launch's first stamp, and its start
// relative to the factorisation's first stamp
static void chol_stamps_dump(int n) {
  std::vector<unsigned long long> h((size_t)3 * kStampCb * kStampWg * 8);
  if (hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_stamp), h.size() * 8) != hipSuccess) return;
  const int nblk = std::min((n + NB - 1) / NB, kStampCb);
  unsigned long long t0 = ~0ull;
  for (unsigned long long v : h)
    if (v && v < t0) t0 = v;
  const char* kinds[3] = {"col+panel", "strip", "bulk"};
  for (int kind = 0; kind < 3; ++kind)
    for (int cb = 0; cb < nblk; ++cb) {
      const unsigned long long* base = h.data() + ((size_t)kind * kStampCb + cb) * kStampWg * 8;
      std::vector<double> ph[8];
      unsigned long long s0 = ~0ull;
      for (int wg = 0; wg < kStampWg; ++wg)
        if (base[wg * 8] && base[wg * 8] < s0) s0 = base[wg * 8];
      if (s0 == ~0ull) continue;
      int nwg = 0;
      for (int wg = 0; wg < kStampWg; ++wg) {
        if (!base[wg * 8]) continue;
        ++nwg;
        for (int p = 0; p < 8; ++p)
          if (base[wg * 8 + p] >= s0) ph[p].push_back((base[wg * 8 + p] - s0) * 0.01);
      }
      fprintf(stderr, "stamps %-9s cb %3d at %8.1f us, %3d wgs:", kinds[kind], cb, (s0 - t0) * 0.01, nwg);
      for (int p = 0; p < 8; ++p) {
        if (ph[p].empty()) continue;
        std::sort(ph[p].begin(), ph[p].end());
        fprintf(stderr, "  p%d %.1f/%.1f", p, ph[p][ph[p].size() / 2], ph[p].back());
      }
      if (kind == 0) {
        const unsigned long long* w0 = base;  // work-group 0: the diagonal tile and the factor
        fprintf(stderr, "  | wg0:");
        for (int p = 0; p < 6; ++p)
          if (w0[p] >= s0) fprintf(stderr, " %.1f", (w0[p] - s0) * 0.01);
      }
      fprintf(stderr, "\n");
    }
}
#endif
int chol_factor_solve(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y, int* d_flag) {
#ifdef DAB_CHOL_STAMPS
  static int calls = 0;
  if (++calls == 4) {
    (void)hipStreamSynchronize(s);
    const int rc = chol_build(c, s, n, A, lda, y, d_flag, true);
    (void)hipStreamSynchronize(s);
    chol_stamps_dump(n);
    return rc;
  }
#endif
  return chol_build(c, s, n, A, lda, y, d_flag, true);
}
// the scratch and the captured graph of a factorisation of this shape and these buffers,
// without running it (the solve's set-up, so its first LM iteration does not capture)
int chol_prepare(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y, int* d_flag) {
  return chol_build(c, s, n, A, lda, y, d_flag, false);
}
static int chol_build(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y, int* d_flag, bool launch) {
  if (n <= 0) return 0;
  const int nblk = (n + NB - 1) / NB;
  if ((size_t)nblk > c->nblk_alloc) {
    if (c->exec) (void)hipGraphExecDestroy(c->exec);
    c->exec = nullptr;
    for (void* p : {(void*)c->blk, (void*)c->pready}) c->mem.drop(p);
    c->blk = nullptr;
    c->pready = nullptr;
    if (c->mem.alloc(&c->blk, (size_t)kBlk * nblk) != 0) return -2;
    if (c->mem.alloc(&c->pready, (size_t)nblk) != 0) return -2;
    c->nblk_alloc = nblk;
  }
  if (!c->side && !(c->side = stream_take(c->device))) return -3;
  if (!c->bar && c->mem.alloc(&c->bar, 1) != 0) return -2;
  while ((int)c->ev_panel.size() < nblk) {
    hipEvent_t a, b, d;
    if (hipEventCreateWithFlags(&a, hipEventDisableTiming) != hipSuccess) return -3;
    if (hipEventCreateWithFlags(&b, hipEventDisableTiming) != hipSuccess) return -3;
    if (hipEventCreateWithFlags(&d, hipEventDisableTiming) != hipSuccess) return -3;
    c->ev_panel.push_back(a);
    c->ev_bulk.push_back(b);
    c->ev_strip.push_back(d);
  }
  // small systems launch directly: a graph's instantiation (~5 ms measured) costs more than
  // the host launches it saves over a whole solve (n = 264, 5 blocks: ~20 launches)
  if (c->nograph || nblk < c->graph_min) {  // nograph: debugging aid
    if (launch) {
      enqueue_factor_solve(c, s, n, A, lda, y, d_flag);
    }
    return 0;
  }
  const bool same = c->exec && c->g_n == n && c->g_lda == lda && c->g_A == A && c->g_y == y && c->g_flag == d_flag;
  if (!same) {
    if (c->exec) (void)hipGraphExecDestroy(c->exec);
    c->exec = nullptr;
    hipGraph_t g = nullptr;
    if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) return -3;
    enqueue_factor_solve(c, s, n, A, lda, y, d_flag);
    if (hipStreamEndCapture(s, &g) != hipSuccess) return -3;
    const hipError_t e = hipGraphInstantiate(&c->exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) {
      c->exec = nullptr;
      return -3;
    }
    c->g_n = n;
    c->g_lda = lda;
    c->g_A = A;
    c->g_y = y;
    c->g_flag = d_flag;
  }
  if (!launch) return 0;
  if (hipGraphLaunch(c->exec, s) != hipSuccess) return -3;
  return 0;
}

static void enqueue_back_substitution(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y,
                                      int* d_flag, bool y_filled);
static void enqueue_factor_solve_v1(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y,
                                    int* d_flag);
// Panel PAIRS with lookahead. Chain stream s, per pair (b, b+1): [wait the previous pair's
// bulk] column b+1 with panel b -> panel b+1 -> column b+2 with panels b, b+1 -> panel b+2;
// bulk stream s2: after panel b+1, the rank-128 update of columns >= b+3 (k_syrk_big),
// overlapping the chain. The trailing matrix is streamed once per two panel steps. Then
// the back substitution in one launch (k_trsv_back_all).
static void enqueue_factor_solve(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y,
                                 int* d_flag) {
  if (c->v1) {
    enqueue_factor_solve_v1(c, s, n, A, lda, y, d_flag);
    return;
  }
  const int nblk = (n + NB - 1) / NB;
  hipStream_t s2 = c->serial ? s : c->side;  // serial: debugging aid
  auto kb_of = [&](int b) { return std::min(NB, n - b * NB); };
  // every panel after the first follows the column update of its block, which factors the
  // diagonal block (DAB_CHOL_PREFACTOR=0: each panel work-group factors it itself)
  const bool pre = c->prefactor, fuse = pre && c->fuse_panel;
  auto panel = [&](int b) {
    // done inside the column update in front, except for a last block shorter than NB,
    // whose rows below (the rhs row) sit in the diagonal tile
    if (fuse && b > 0 && kb_of(b) == NB) return;
    const int k = b * NB, kb = kb_of(b);
    const int r0 = k + kb, r1 = n + 1;  // includes the rhs row n
    const int grid = std::max(1, (r1 - r0 + NB - 1) / NB);
    // the first panel also fills y (pending) and zeroes the fused steps' flags
    const bool first = b == 0;
    k_panel<<<grid, kThreads, 0, s>>>(A, lda, k, kb, r0, r1, c->blk + (size_t)b * kBlk, d_flag, pre && b > 0,
                                      first ? y : nullptr, first ? n : 0, first && fuse ? c->pready : nullptr,
                                      first && fuse ? nblk : 0);
  };
  // column block cb (rows >= its first row, through the rhs row) with panel columns [k, k + kk)
  auto col = [&](int cb, int k, int kk) {
    const int r0 = cb * NB, m = n + 1 - r0;
    if (m <= 1) return;
    const int nt = (m + NB - 1) / NB;
    if (pre)
      k_syrk_mfma<true><<<nt, kThreads, 0, s>>>(A, lda, r0, m, k, kk, 1, nt, c->blk + (size_t)cb * kBlk, kb_of(cb),
                                                d_flag, fuse ? c->pready + cb : nullptr);
    else
      k_syrk_mfma<false><<<nt, kThreads, 0, s>>>(A, lda, r0, m, k, kk, 1, nt);
  };
  panel(0);
  // groups of R = c->group panels (2: the pairs). Within a group the chain updates column c
  // with the group's panels [b, c) itself; after the group's last panel but one, the bulk
  // update applies all R panels to the columns >= b + R + 1 while the chain does column b + R.
  const int R = std::max(2, c->group);
  int pending = -1;  // group whose bulk update is still running on s2
  // strip (round 5): the bulk's first block column (the next group's first column) is a
  // launch of its own on s2, so the chain's next column update waits for it only and runs
  // beside the rest of the bulk instead of alone after it; the group's last column waits
  // for the whole bulk. n = 5994: 5.63 -> 4.95-5.0 ms (scripts/runs/r05ai.sh)
  const bool strip = c->strip;
  for (int b = 0; b + 1 < nblk; b += R) {
    const int prev = pending;
    pending = -1;
    if (prev >= 0) (void)hipStreamWaitEvent(s, strip ? c->ev_strip[prev] : c->ev_bulk[prev], 0);
    const int cend = std::min(b + R, nblk);  // first column past the group's panels
    for (int cc = b + 1; cc < cend; ++cc) {  // every panel before the last is NB wide
      if (strip && prev >= 0 && cc > b + 1) (void)hipStreamWaitEvent(s, c->ev_bulk[prev], 0);
      col(cc, b * NB, (cc - b) * NB);
      panel(cc);
    }
    if (strip && prev >= 0) (void)hipStreamWaitEvent(s, c->ev_bulk[prev], 0);
    if (cend >= nblk) break;  // the group ended at the last panel (its solve covered the rhs row)
    const int kk = (cend - b) * NB;
    const int c0 = (cend + (strip ? 2 : 1)) * NB, m = n + 1 - c0;
    const int cs0 = (cend + 1) * NB, ms = n + 1 - cs0;
    if (m > 1 || (strip && ms > 1)) {
      (void)hipEventRecord(c->ev_panel[b], s);
      (void)hipStreamWaitEvent(s2, c->ev_panel[b], 0);
      if (strip && ms > 1) {
        const int nts = (ms + NB - 1) / NB;
        k_syrk_mfma<false><<<nts, kThreads, 0, s2>>>(A, lda, cs0, ms, b * NB, kk, 1, nts);
        (void)hipEventRecord(c->ev_strip[b], s2);
      }
      if (m > 1) {
        const int t2 = (m + TB - 1) / TB, ntb = t2 * (t2 + 1) / 2;
        // the bulk grid leaves CUs free for the panel chain (its dependent MFMA chain would
        // queue behind the bulk's MFMAs on a shared CU)
        const int g = std::min(ntb, c->bulk_grid > 0 ? c->bulk_grid : ntb);
        k_syrk_big<16, 4><<<g, kBigThreads, 0, s2>>>(A, lda, c0, m, b * NB, kk, ntb);
      }
      (void)hipEventRecord(c->ev_bulk[b], s2);
      if (strip && ms <= 1) (void)hipEventRecord(c->ev_strip[b], s2);
      pending = b;
    }
    col(cend, b * NB, kk);
    panel(cend);
  }
  if (pending >= 0) (void)hipStreamWaitEvent(s, c->ev_bulk[pending], 0);
  enqueue_back_substitution(c, s, n, A, lda, y, d_flag, true);
}

// y_filled: the factorisation's first panel launch set y to the pending pattern
static void enqueue_back_substitution(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y,
                                      int* d_flag, bool y_filled) {
  const int nblk = (n + NB - 1) / NB;
  double* z = A + (size_t)n * lda;
  const int G = std::max(1, std::min(c->ncu / 2, (n + 63) / 64));
  if (c->back_flow && nblk <= G * kMaxOwned) {
    // y_b is pending until its owner stores it (k_trsv_back_flow polls the values themselves)
    if (!y_filled) (void)hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(y), kYPending32, 2 * (size_t)n, s);
    k_trsv_back_flow<<<G, kThreads, 0, s>>>(A, lda, n, nblk, c->blk, z, y, d_flag);
    return;
  }
  (void)hipMemsetAsync(c->bar, 0, sizeof(unsigned), s);
  k_trsv_back_all<<<G, kThreads, 0, s>>>(A, lda, n, nblk, c->blk, z, y, c->bar, d_flag);
}

static void enqueue_factor_solve_v1(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y,
                                    int* d_flag) {
  // Lookahead by one block column. Chain stream s: P(0), then per step b
  // [wait bulk(b-1)] col-update(b) -> P(b+1); bulk stream s2: bulk(b) after P(b). The
  // bulk trailing update of step b overlaps the next panel step.
  const int nblk = (n + NB - 1) / NB;
  hipStream_t s2 = c->serial ? s : c->side;  // serial: debugging aid
  auto panel = [&](int b) {
    const int k = b * NB, kb = (n - k < NB) ? n - k : NB;
    const int r0 = k + kb, r1 = n + 1;  // includes the rhs row n
    const int grid = std::max(1, (r1 - r0 + NB - 1) / NB);
    k_panel<<<grid, kThreads, 0, s>>>(A, lda, k, kb, r0, r1, c->blk + (size_t)b * kBlk, d_flag, 0);
  };
  panel(0);
  bool bulk_prev = false;
  for (int b = 0; b < nblk; ++b) {
    const int k = b * NB, kb = (n - k < NB) ? n - k : NB;
    const int r0 = k + kb, m = n + 1 - r0;
    if (m <= 1 && b + 1 >= nblk) break;
    const int nt = (m + NB - 1) / NB;
    bool bulk = false;
    if (nt > 1) {  // tile columns 1.. of the trailing matrix
      (void)hipEventRecord(c->ev_panel[b], s);
      (void)hipStreamWaitEvent(s2, c->ev_panel[b], 0);
      const int m2 = m - NB, nt2 = (m2 + NB - 1) / NB;
      const int ntb = nt2 * (nt2 + 1) / 2;
      k_syrk_mfma<false><<<std::min(ntb, c->bulk_grid > 0 ? c->bulk_grid : ntb), kThreads, 0, s2>>>(A, lda, r0 + NB, m2, k,
                                                                                         kb, 0, ntb);
      (void)hipEventRecord(c->ev_bulk[b], s2);
      bulk = true;
    }
    if (bulk_prev) (void)hipStreamWaitEvent(s, c->ev_bulk[b - 1], 0);
    if (m > 1) k_syrk_mfma<false><<<nt, kThreads, 0, s>>>(A, lda, r0, m, k, kb, 1, nt);
    if (b + 1 < nblk) panel(b + 1);
    bulk_prev = bulk;
  }
  // join the bulk stream (its last event) before the back substitution
  for (int b = nblk - 1; b >= 0; --b) {
    const int k = b * NB, kb = (n - k < NB) ? n - k : NB;
    const int m = n + 1 - (k + kb), nt = (m + NB - 1) / NB;
    if (nt > 1) {
      (void)hipStreamWaitEvent(s, c->ev_bulk[b], 0);
      break;
    }
  }
  double* z = A + (size_t)n * lda;
  for (int b = nblk - 1; b >= 0; --b) {
    const int k = b * NB, kb = (n - k < NB) ? n - k : NB;
    const int grid = k > 0 ? (k + 63) / 64 : 1;
    k_trsv_back<<<grid, kThreads, 0, s>>>(A, lda, k, kb, c->blk + (size_t)b * kBlk, z, y);
  }
}

// DAB_DEV_GUARD: the canaries after the scratch blocks (the caller has synchronised)
int chol_guard_check(CholCtx* c, const char* where, std::string* first) {
  return c ? c->mem.guard_check(where, first) : 0;
}
Dev* chol_mem(CholCtx* c) { return c ? &c->mem : nullptr; }

// Loads this translation unit's code object on the current device now: otherwise the first
// launch of any of its kernels pays for it (10-40 ms, inside a process's first LM iteration).
void warm_chol() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(k_panel));
}

}  // namespace dab
