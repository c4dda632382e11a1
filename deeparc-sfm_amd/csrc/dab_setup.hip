// dab_setup.hip — dab_set_problem's orderings and reduction tables built on the GPU.
//
// The host passes of dab_solver.hip (the reference path, DAB_SETUP_HOST=1) are stable
// counting sorts and gathers over every observation; at BASELINE config 5 (10M
// observations) they took ~0.7 s per set-up, and the reference's sfm.cc loop re-runs the
// set-up after every filterPoint3d round (sfm.cc:118-127). Here the same orders come from
// rocPRIM's LSD radix sorts — stable, so ties keep input order exactly as the host's
// counting sorts do — and the rest are one-thread-per-element gather / scatter passes or
// one-block-per-chunk passes with a fixed in-block order. Every output is bitwise the
// host path's (tests/test_gpu_setup.py).
#include <hip/hip_runtime.h>

#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_reduce.hpp>
#include <rocprim/device/device_run_length_encode.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_select.hpp>

#include "dab_setup.h"

namespace dab {

namespace {
constexpr int kSuBlock = 256;
inline unsigned su_grid(long long n) { return (unsigned)std::max(1LL, std::min((n + kSuBlock - 1) / kSuBlock, 1LL << 20)); }

// block-wide sum of one int per thread (256 threads), result valid in every thread
__device__ __forceinline__ int block_sum(int x, int* lds) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  if (lane == 0) lds[w] = x;
  __syncthreads();
  int t = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += lds[i];
  __syncthreads();
  return t;
}
}  // namespace

// ---- rocPRIM wrappers ----
int su_sort_pairs(void* tmp, size_t* tmp_bytes, const int* kin, int* kout, const int* vin, int* vout, int n,
                  int end_bit, hipStream_t s) {
  return rocprim::radix_sort_pairs(tmp, *tmp_bytes, kin, kout, vin, vout, (unsigned)n, 0u, (unsigned)end_bit, s) ==
                 hipSuccess ? 0 : -1;
}
int su_exclusive_scan(void* tmp, size_t* tmp_bytes, const int* in, int* out, int n, hipStream_t s) {
  return rocprim::exclusive_scan(tmp, *tmp_bytes, in, out, 0, (size_t)n, rocprim::plus<int>(), s) == hipSuccess ? 0
                                                                                                             : -1;
}
int su_max(void* tmp, size_t* tmp_bytes, const int* in, int* out, int n, hipStream_t s) {
  return rocprim::reduce(tmp, *tmp_bytes, in, out, 0, (size_t)n, rocprim::maximum<int>(), s) == hipSuccess ? 0 : -1;
}
int su_select_flagged_i(void* tmp, size_t* tmp_bytes, const int* in, const unsigned char* flags, int* out,
                        int* count, int n, hipStream_t s) {
  return rocprim::select(tmp, *tmp_bytes, in, flags, out, count, (size_t)n, s) == hipSuccess ? 0 : -1;
}
int su_rle(void* tmp, size_t* tmp_bytes, const int* in, int* unique, int* counts, int* nruns, int n, hipStream_t s) {
  return rocprim::run_length_encode(tmp, *tmp_bytes, in, (size_t)n, unique, counts, nruns, s) == hipSuccess ? 0 : -1;
}

// ---- (1) counts ----
__global__ __launch_bounds__(kSuBlock) void k_su_count(int N, const int* __restrict__ obs_point,
                                                       const int* __restrict__ obs_ext0,
                                                       const int* __restrict__ obs_ext1,
                                                       const int* __restrict__ obs_intr, int num_points, int num_ext,
                                                       int num_intr, int* __restrict__ pcount, int* __restrict__ eref,
                                                       int* __restrict__ flags) {
  // referenced extrinsics marked in LDS first (10M observations over ~100 extrinsics would
  // otherwise store to the same few lines from every wave)
  __shared__ int seref[4096];
  const bool lds = num_ext <= 4096;
  if (lds)
    for (int i = threadIdx.x; i < num_ext; i += blockDim.x) seref[i] = 0;
  __syncthreads();
  int bad = 0, comp = 0;
  for (long long o = blockIdx.x * (long long)blockDim.x + threadIdx.x; o < N; o += (long long)gridDim.x * blockDim.x) {
    const int pt = obs_point[o], e0 = obs_ext0[o], e1 = obs_ext1[o], ii = obs_intr[o];
    if (pt < 0 || pt >= num_points || e0 < 0 || e0 >= num_ext || e1 < -1 || e1 >= num_ext || ii < 0 ||
        ii >= num_intr) {
      bad = 1;
      continue;
    }
    atomicAdd(&pcount[pt], 1);
    if (lds) seref[e0] = 1;
    else eref[e0] = 1;
    if (e1 >= 0) {
      comp = 1;
      if (lds) seref[e1] = 1;
      else eref[e1] = 1;
    }
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flags, 1);
  if (__any(comp) && (threadIdx.x & 63) == 0) atomicOr(flags, 2);
  __syncthreads();
  if (lds)
    for (int i = threadIdx.x; i < num_ext; i += blockDim.x)
      if (seref[i]) eref[i] = 1;
}
void su_count(hipStream_t s, int N, const int* obs_point, const int* obs_ext0, const int* obs_ext1,
              const int* obs_intr, int num_points, int num_ext, int num_intr, int* pcount, int* eref, int* flags) {
  if (N <= 0) return;
  k_su_count<<<std::min(su_grid(N), 2048u), kSuBlock, 0, s>>>(N, obs_point, obs_ext0, obs_ext1, obs_intr, num_points,
                                                               num_ext, num_intr, pcount, eref, flags);
}

// ---- (2), (3) device point order ----
__global__ __launch_bounds__(kSuBlock) void k_su_point_keys(int n, const int* __restrict__ pcount,
                                                            const int* __restrict__ maxcount, int* __restrict__ keys,
                                                            int* __restrict__ vals, int* __restrict__ nref) {
  __shared__ int red[kSuBlock / 64];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int mc = *maxcount;
  int ref = 0;
  if (i < n) {
    const int c = pcount[i];
    ref = c > 0;
    keys[i] = ref ? mc - c : mc + 1;  // count descending; unreferenced points last
    vals[i] = i;
  }
  const int t = block_sum(ref, red);
  if (threadIdx.x == 0 && t) atomicAdd(nref, t);
}
void su_point_keys(hipStream_t s, int num_points, const int* pcount, const int* maxcount, int* keys, int* vals,
                   int* nref) {
  if (num_points <= 0) return;
  k_su_point_keys<<<su_grid(num_points), kSuBlock, 0, s>>>(num_points, pcount, maxcount, keys, vals, nref);
}

__global__ void k_su_point_local(int NP, const int* __restrict__ pt_of, const int* __restrict__ pcount,
                                 int* __restrict__ pt_local, int* __restrict__ lcount) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l < NP) {
    const int p = pt_of[l];
    pt_local[p] = l;
    lcount[l] = pcount[p];
  } else if (l == NP) {
    lcount[NP] = 0;  // the scan's last element: cnt[NP] = N
  }
}
void su_point_local(hipStream_t s, int NP, const int* pt_of, const int* pcount, int* pt_local, int* lcount) {
  k_su_point_local<<<su_grid(NP + 1), kSuBlock, 0, s>>>(NP, pt_of, pcount, pt_local, lcount);
}

// ---- (4) observation keys ----
__global__ void k_su_obs_keys(int N, const int* __restrict__ obs_point, const int* __restrict__ pt_local,
                              int* __restrict__ keys, int* __restrict__ vals) {
  for (long long o = blockIdx.x * (long long)blockDim.x + threadIdx.x; o < N; o += (long long)gridDim.x * blockDim.x) {
    keys[o] = pt_local[obs_point[o]];
    vals[o] = (int)o;
  }
}
void su_obs_keys(hipStream_t s, int N, const int* obs_point, const int* pt_local, int* keys, int* vals) {
  if (N > 0) k_su_obs_keys<<<su_grid(N), kSuBlock, 0, s>>>(N, obs_point, pt_local, keys, vals);
}

// ---- (5) slices ----
__global__ void k_su_slice_len(int nslice, int NP, const int* __restrict__ lcount, int* __restrict__ slen) {
  const int sl = blockIdx.x * blockDim.x + threadIdx.x;
  if (sl < nslice) slen[sl] = 64 * lcount[64 * sl];  // the slice's first point has its longest track
  else if (sl == nslice) slen[sl] = 0;
}
void su_slice_len(hipStream_t s, int nslice, int NP, const int* lcount, int* slen) {
  k_su_slice_len<<<su_grid(nslice + 1), kSuBlock, 0, s>>>(nslice, NP, lcount, slen);
}

// ---- (6) SELL-64 slots ----
// one thread per (slice, lane): the lane's point's observations in caller order, then the
// slice's padding. Lanes of a wave write 64 consecutive slots per row (coalesced).
__global__ void k_su_slots(int NP, int nslice, const int* __restrict__ slice_off, const int* __restrict__ cnt,
                           const int* __restrict__ lcount, const int* __restrict__ by_pt,
                           const int* __restrict__ obs_ext0, const int* __restrict__ obs_ext1,
                           const int* __restrict__ obs_intr, const double* __restrict__ obs_xy,
                           const int* __restrict__ ext_col, int4* __restrict__ obs_idx,
                           double2* __restrict__ xy_out, int* __restrict__ perm, int* __restrict__ ne_out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 64 * nslice) {
    if (t == 64 * nslice) ne_out[NP] = 0;
    return;
  }
  const int sl = t >> 6, lane = t & 63, pt = t;
  const int rows = (slice_off[sl + 1] - slice_off[sl]) >> 6;
  const int len = pt < NP ? lcount[pt] : 0;
  const int base = pt < NP ? cnt[pt] : 0;
  int ne = 0;
  for (int k = 0; k < rows; ++k) {
    const int slot = slice_off[sl] + 64 * k + lane;
    if (k < len) {
      const int o = by_pt[base + k];
      const int e0 = obs_ext0[o], e1 = obs_ext1[o];
      obs_idx[slot] = make_int4(pt, e0, e1, obs_intr[o]);
      xy_out[slot] = make_double2(obs_xy[2 * (size_t)o], obs_xy[2 * (size_t)o + 1]);
      perm[slot] = o;
      ne += ext_col[e0] >= 0;
      ne += e1 >= 0 && ext_col[e1] >= 0;
    } else {
      obs_idx[slot] = make_int4(-1, 0, -1, 0);
      xy_out[slot] = make_double2(0.0, 0.0);
      perm[slot] = -1;
    }
  }
  if (pt < NP) ne_out[pt] = ne;
}
void su_slots(hipStream_t s, int NP, int nslice, const int* slice_off, const int* cnt, const int* lcount,
              const int* by_pt, const int* obs_ext0, const int* obs_ext1, const int* obs_intr, const double* obs_xy,
              const int* ext_col, int4* obs_idx, double2* obs_xy_out, int* perm, int* ne) {
  k_su_slots<<<su_grid(64LL * nslice + 1), kSuBlock, 0, s>>>(NP, nslice, slice_off, cnt, lcount, by_pt, obs_ext0,
                                                             obs_ext1, obs_intr, obs_xy, ext_col, obs_idx, obs_xy_out,
                                                             perm, ne);
}

// ---- (7) entries ----
__global__ void k_su_entries(int NP, const int* __restrict__ slice_off, const int* __restrict__ lcount,
                             const int4* __restrict__ obs_idx, const int* __restrict__ ext_col,
                             const int* __restrict__ pt_ent_ptr, int* __restrict__ ent_os, int* __restrict__ ent_cam,
                             int* __restrict__ ent_pt) {
  const int pt = blockIdx.x * blockDim.x + threadIdx.x;
  if (pt >= NP) return;
  const int sl = pt >> 6, lane = pt & 63;
  int q = pt_ent_ptr[pt];
  for (int k = 0; k < lcount[pt]; ++k) {
    const int s2 = slice_off[sl] + 64 * k + lane;
    const int4 id = obs_idx[s2];
#pragma unroll
    for (int slot = 0; slot < 2; ++slot) {
      const int ex = slot ? id.z : id.y;
      if (ex < 0) continue;
      const int c = ext_col[ex];
      if (c < 0) continue;
      ent_os[q] = 2 * s2 + slot;
      ent_cam[q] = c;
      ent_pt[q] = pt;
      ++q;
    }
  }
}
void su_entries(hipStream_t s, int NP, const int* slice_off, const int* lcount, const int4* obs_idx,
                const int* ext_col, const int* pt_ent_ptr, int* ent_os, int* ent_cam, int* ent_pt) {
  if (NP > 0)
    k_su_entries<<<su_grid(NP), kSuBlock, 0, s>>>(NP, slice_off, lcount, obs_idx, ext_col, pt_ent_ptr, ent_os, ent_cam,
                                                  ent_pt);
}

// ---- (8) key boundaries ----
__global__ void k_su_bounds(int n, const int* __restrict__ key, int nkeys, int* __restrict__ start) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int k = key[i], kp = i == 0 ? -1 : key[i - 1];
  for (int c = kp + 1; c <= k && c <= nkeys; ++c) start[c] = i;
  if (i == n - 1)
    for (int c = k + 1; c <= nkeys; ++c) start[c] = n;
}
void su_bounds(hipStream_t s, int n, const int* sorted_keys, int nkeys, int* start) {
  if (n > 0) k_su_bounds<<<su_grid(n), kSuBlock, 0, s>>>(n, sorted_keys, nkeys, start);
}

// ---- (9) camera-major copies ----
__global__ void k_su_camera_major(int NE, const int* __restrict__ cam_ent, const int* __restrict__ ent_pt,
                                  const int* __restrict__ ent_os, const int4* __restrict__ obs_idx,
                                  const double2* __restrict__ obs_xy, int* __restrict__ ent_pos,
                                  int* __restrict__ cm_pt, int4* __restrict__ cm_idx, double2* __restrict__ cm_xy,
                                  int slot_bit) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < NE; i += (long long)gridDim.x * blockDim.x) {
    const int e = cam_ent[i];
    ent_pos[e] = (int)i;
    cm_pt[i] = ent_pt[e];
    const int os = ent_os[e], s2 = os >> 1;
    int4 id = obs_idx[s2];
    if (os & 1) id.w |= slot_bit;
    cm_idx[i] = id;
    cm_xy[i] = obs_xy[s2];
  }
}
void su_camera_major(hipStream_t s, int NE, const int* cam_ent, const int* ent_pt, const int* ent_os,
                     const int4* obs_idx, const double2* obs_xy, int* ent_pos, int* cm_pt, int4* cm_idx,
                     double2* cm_xy) {
  constexpr int kSlotBitHere = 1 << 30;  // dab_kernels.h kSlotBit
  if (NE > 0)
    k_su_camera_major<<<su_grid(NE), kSuBlock, 0, s>>>(NE, cam_ent, ent_pt, ent_os, obs_idx, obs_xy, ent_pos, cm_pt,
                                                       cm_idx, cm_xy, kSlotBitHere);
}

// ---- (10) runs ----
__global__ void k_su_runs(int NE, const int* __restrict__ pos_cam, const int* __restrict__ cm_pt,
                          int* __restrict__ run) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < NE; i += (long long)gridDim.x * blockDim.x) {
    const int c = pos_cam[i], p = cm_pt[i];
    const bool start = i == 0 || pos_cam[i - 1] != c || cm_pt[i - 1] != p;
    int len = 0;
    if (start) {
      long long j = i + 1;
      while (j < NE && pos_cam[j] == c && cm_pt[j] == p) ++j;
      len = (int)(j - i);
    }
    run[i] = len;
  }
}
void su_runs(hipStream_t s, int NE, const int* pos_cam, const int* cm_pt, int* run) {
  if (NE > 0) k_su_runs<<<su_grid(NE), kSuBlock, 0, s>>>(NE, pos_cam, cm_pt, run);
}

// ---- (11) per-chunk passes (one block per chunk) ----
__global__ __launch_bounds__(kSuBlock) void k_su_chunk_runs(const int* __restrict__ chunk_beg,
                                                            const int* __restrict__ run, int* __restrict__ run_cnt,
                                                            int nchunk) {
  __shared__ int red[kSuBlock / 64];
  const int q = blockIdx.x;
  int n = 0;
  for (int i = chunk_beg[q] + threadIdx.x; i < chunk_beg[q + 1]; i += blockDim.x) n += run[i] > 0;
  const int t = block_sum(n, red);
  if (threadIdx.x == 0) run_cnt[q] = t;
  if (q == 0 && threadIdx.x == 0) run_cnt[nchunk] = 0;
}
void su_chunk_runs(hipStream_t s, int nchunk, const int* chunk_beg, const int* run, int* run_cnt) {
  if (nchunk > 0) k_su_chunk_runs<<<nchunk, kSuBlock, 0, s>>>(chunk_beg, run, run_cnt, nchunk);
}

// records of the chunk's runs in position order: tiles of 256 positions, a block-wide
// exclusive scan of the run-start flags gives each record's place
__global__ __launch_bounds__(kSuBlock) void k_su_chunk_run_rec(const int* __restrict__ chunk_beg,
                                                               const int* __restrict__ run,
                                                               const int* __restrict__ cm_pt,
                                                               const int* __restrict__ pos_cam,
                                                               const int* __restrict__ run_beg,
                                                               int4* __restrict__ run_rec) {
  __shared__ int pre[kSuBlock];
  const int q = blockIdx.x;
  int base = run_beg[q];
  for (int t0 = chunk_beg[q]; t0 < chunk_beg[q + 1]; t0 += blockDim.x) {
    const int i = t0 + (int)threadIdx.x;
    const int f = i < chunk_beg[q + 1] && run[i] > 0;
    pre[threadIdx.x] = f;
    __syncthreads();
    for (int o = 1; o < (int)blockDim.x; o <<= 1) {  // inclusive Hillis-Steele scan
      const int v = threadIdx.x >= (unsigned)o ? pre[threadIdx.x - o] : 0;
      __syncthreads();
      pre[threadIdx.x] += v;
      __syncthreads();
    }
    if (f) run_rec[base + pre[threadIdx.x] - 1] = make_int4(i, run[i], cm_pt[i], pos_cam[i]);
    base += pre[blockDim.x - 1];
    __syncthreads();
  }
}
void su_chunk_run_rec(hipStream_t s, int nchunk, const int* chunk_beg, const int* run, const int* cm_pt,
                      const int* pos_cam, const int* run_beg, int4* run_rec) {
  if (nchunk > 0) k_su_chunk_run_rec<<<nchunk, kSuBlock, 0, s>>>(chunk_beg, run, cm_pt, pos_cam, run_beg, run_rec);
}

__global__ __launch_bounds__(kSuBlock) void k_su_chunk_uni(const int* __restrict__ chunk_beg,
                                                           const int4* __restrict__ cm_idx, int slot_bit,
                                                           int2* __restrict__ chunk_uni) {
  const int q = blockIdx.x;
  const int4 first = cm_idx[chunk_beg[q]];
  int uni = first.z < 0 && !(first.w & slot_bit);
  for (int i = chunk_beg[q] + threadIdx.x; uni && i < chunk_beg[q + 1]; i += blockDim.x) {
    const int4 id = cm_idx[i];
    uni = id.z < 0 && id.y == first.y && id.w == first.w;
  }
  uni = __syncthreads_and(uni);
  if (threadIdx.x == 0) chunk_uni[q] = uni ? make_int2(first.y, first.w) : make_int2(-1, -1);
}
void su_chunk_uni(hipStream_t s, int nchunk, const int* chunk_beg, const int4* cm_idx, int slot_bit, int2* chunk_uni) {
  if (nchunk > 0) k_su_chunk_uni<<<nchunk, kSuBlock, 0, s>>>(chunk_beg, cm_idx, slot_bit, chunk_uni);
}

// ---- (12), (13) pair-major copy ----
__global__ __launch_bounds__(kSuBlock) void k_su_cross_keys(int NS, const int4* __restrict__ obs_idx,
                                                            const int* __restrict__ ext_col, int NC,
                                                            int* __restrict__ keys, int* __restrict__ vals,
                                                            int* __restrict__ nvalid) {
  __shared__ int red[kSuBlock / 64];
  const int s2 = blockIdx.x * blockDim.x + threadIdx.x;
  int valid = 0;
  if (s2 < NS) {
    const int4 id = obs_idx[s2];
    int key = NC * NC;  // sentinel: sorted past every pair
    if (id.z >= 0 && id.x >= 0) {
      const int c0 = ext_col[id.y], c1 = ext_col[id.z];
      if (c0 >= 0 && c1 >= 0) {
        key = c0 * NC + c1;
        valid = 1;
      }
    }
    keys[s2] = key;
    vals[s2] = s2;
  }
  const int t = block_sum(valid, red);
  if (threadIdx.x == 0 && t) atomicAdd(nvalid, t);
}
void su_cross_keys(hipStream_t s, int NS, const int4* obs_idx, const int* ext_col, int NC, int* keys, int* vals,
                   int* nvalid) {
  if (NS > 0) k_su_cross_keys<<<su_grid(NS), kSuBlock, 0, s>>>(NS, obs_idx, ext_col, NC, keys, vals, nvalid);
}

__global__ void k_su_cross_copy(int n, const int* __restrict__ slots, const int4* __restrict__ obs_idx,
                                const double2* __restrict__ obs_xy, int4* __restrict__ x_idx,
                                double2* __restrict__ x_xy, unsigned char* __restrict__ touched) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int s2 = slots[i];
    const int4 id = obs_idx[s2];
    x_idx[i] = id;
    x_xy[i] = obs_xy[s2];
    if (touched) touched[id.x] = 1;
  }
}
void su_cross_copy(hipStream_t s, int n, const int* slots, const int4* obs_idx, const double2* obs_xy, int4* x_idx,
                   double2* x_xy, unsigned char* touched) {
  if (n > 0) k_su_cross_copy<<<su_grid(n), kSuBlock, 0, s>>>(n, slots, obs_idx, obs_xy, x_idx, x_xy, touched);
}

__global__ __launch_bounds__(kSuBlock) void k_su_count_flags(int n, const unsigned char* __restrict__ f,
                                                             int* __restrict__ count) {
  __shared__ int red[kSuBlock / 64];
  int c = 0;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    c += f[i] != 0;
  const int t = block_sum(c, red);
  if (threadIdx.x == 0 && t) atomicAdd(count, t);
}
void su_count_flags(hipStream_t s, int n, const unsigned char* flags, int* count) {
  if (n > 0) k_su_count_flags<<<std::min(su_grid(n), 2048u), kSuBlock, 0, s>>>(n, flags, count);
}

// ---- (14b) one intrinsic per pair ----
// k_eval_pair reads the arc, ring and intrinsic tables of a chunk once (uniform values)
// when every pair-major record of one (arc, ring) pair names the same intrinsic; count the
// neighbours in one pair that differ (0: the fast form applies)
__global__ __launch_bounds__(kSuBlock) void k_su_pair_intr(int n, const int4* __restrict__ x_idx,
                                                           int* __restrict__ count) {
  __shared__ int red[kSuBlock / 64];
  int c = 0;
  for (long long i = 1 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int4 a = x_idx[i - 1], b = x_idx[i];
    c += a.y == b.y && a.z == b.z && a.w != b.w;
  }
  const int t = block_sum(c, red);
  if (threadIdx.x == 0 && t) atomicAdd(count, t);
}
void su_pair_intr(hipStream_t s, int n, const int4* x_idx, int* count) {
  if (n > 1) k_su_pair_intr<<<std::min(su_grid(n), 2048u), kSuBlock, 0, s>>>(n, x_idx, count);
}

// ---- (15) unpaired entries ----
__global__ void k_su_unpaired(int NE, const int4* __restrict__ cm_idx, const int* __restrict__ ext_col,
                              unsigned char* __restrict__ flags, int* __restrict__ flags_i) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i <= NE; i += (long long)gridDim.x * blockDim.x) {
    int u = 0;
    if (i < NE) {
      const int4 id = cm_idx[i];
      u = !(id.z >= 0 && ext_col[id.y] >= 0 && ext_col[id.z] >= 0);
      flags[i] = (unsigned char)u;
    }
    flags_i[i] = u;  // [NE + 1]: the scan's last element
  }
}
void su_unpaired_flags(hipStream_t s, int NE, const int4* cm_idx, const int* ext_col, unsigned char* flags,
                       int* flags_i) {
  k_su_unpaired<<<su_grid(NE + 1), kSuBlock, 0, s>>>(NE, cm_idx, ext_col, flags, flags_i);
}
__global__ void k_su_gather_cm(int n, const int* __restrict__ sel, const int4* __restrict__ cm_idx,
                               const double2* __restrict__ cm_xy, int4* __restrict__ out_idx,
                               double2* __restrict__ out_xy) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const int j = sel[i];
    out_idx[i] = cm_idx[j];
    out_xy[i] = cm_xy[j];
  }
}
void su_gather_cm(hipStream_t s, int n, const int* sel, const int4* cm_idx, const double2* cm_xy, int4* out_idx,
                  double2* out_xy) {
  if (n > 0) k_su_gather_cm<<<su_grid(n), kSuBlock, 0, s>>>(n, sel, cm_idx, cm_xy, out_idx, out_xy);
}

// ---- (16), (17) ----
__global__ void k_su_obs_e(int NS, const int4* __restrict__ obs_idx, int* __restrict__ obs_e) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < NS; i += (long long)gridDim.x * blockDim.x) {
    const int4 id = obs_idx[i];
    obs_e[i] = id.x >= 0 ? (id.y | (id.w << 16)) : -1;
  }
}
void su_obs_e(hipStream_t s, int NS, const int4* obs_idx, int* obs_e) {
  if (NS > 0) k_su_obs_e<<<su_grid(NS), kSuBlock, 0, s>>>(NS, obs_idx, obs_e);
}
__global__ void k_su_points(int NP, const int* __restrict__ pt_of, const double* __restrict__ raw,
                            double* __restrict__ points) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 3 * NP) return;
  const int l = i / 3, k = i - 3 * l;
  points[i] = raw[3 * (size_t)pt_of[l] + k];
}
void su_points(hipStream_t s, int NP, const int* pt_of, const double* raw_points, double* points) {
  if (NP > 0) k_su_points<<<su_grid(3LL * NP), kSuBlock, 0, s>>>(NP, pt_of, raw_points, points);
}
__global__ void k_su_iota(int n, int* __restrict__ out) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = (int)i;
}
void su_iota(hipStream_t s, int n, int* out) {
  if (n > 0) k_su_iota<<<su_grid(n), kSuBlock, 0, s>>>(n, out);
}

// gather out[c] = in[idx[c]] for c < n (small tables read back to the host)
__global__ void k_su_gather_at(int n, const int* __restrict__ idx, const int* __restrict__ in, int* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < n) out[c] = in[idx[c]];
}
void su_gather_at(hipStream_t s, int n, const int* idx, const int* in, int* out) {
  if (n > 0) k_su_gather_at<<<su_grid(n), kSuBlock, 0, s>>>(n, idx, in, out);
}

void warm_setup() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(k_su_count));
}

// ---- (18) explicit-Schur pair tables (build_schur_tables, large camera sets) ----
// ordered entry pairs (e, f) of one point with cam(e) >= cam(f), generated per point in
// (e, f) order: the host path's order before its stable sort by block key
__global__ __launch_bounds__(kSuBlock) void k_su_pair_count(int NP, const int* __restrict__ ptr,
                                                            const int* __restrict__ cam, int* __restrict__ cnt,
                                                            unsigned long long* __restrict__ total) {
  __shared__ int red[kSuBlock / 64];
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  int c = 0;
  if (p < NP) {
    const int b = ptr[p], e = ptr[p + 1];
    for (int i = b; i < e; ++i) {
      const int ci = cam[i];
      for (int j = b; j < e; ++j) c += ci >= cam[j];
    }
    cnt[p] = c;
  }
  const int t = block_sum(c, red);
  if (threadIdx.x == 0 && t) atomicAdd(total, (unsigned long long)t);  // integer: order-free
}
void su_pair_count(hipStream_t s, int NP, const int* pt_ent_ptr, const int* ent_cam, int* cnt,
                   unsigned long long* total) {
  if (NP > 0) k_su_pair_count<<<su_grid(NP), kSuBlock, 0, s>>>(NP, pt_ent_ptr, ent_cam, cnt, total);
}
__global__ void k_su_pair_gen(int NP, const int* __restrict__ ptr, const int* __restrict__ cam,
                              const int* __restrict__ poff, int NC, int* __restrict__ keys, int* __restrict__ vals,
                              int2* __restrict__ ef) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= NP) return;
  const int b = ptr[p], e = ptr[p + 1];
  int o = poff[p];
  for (int i = b; i < e; ++i) {
    const int ci = cam[i];
    for (int j = b; j < e; ++j) {
      const int cj = cam[j];
      if (ci < cj) continue;
      keys[o] = ci * NC + cj;
      vals[o] = o;
      ef[o] = make_int2(i, j);
      ++o;
    }
  }
}
void su_pair_gen(hipStream_t s, int NP, const int* pt_ent_ptr, const int* ent_cam, const int* poff, int NC, int* keys,
                 int* vals, int2* ef) {
  if (NP > 0) k_su_pair_gen<<<su_grid(NP), kSuBlock, 0, s>>>(NP, pt_ent_ptr, ent_cam, poff, NC, keys, vals, ef);
}
__global__ void k_su_pair_gather(int n, const int* __restrict__ idx, const int2* __restrict__ ef,
                                 const int* __restrict__ ent_pos, int2* __restrict__ pairs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int2 q = ef[idx[i]];
  pairs[i] = make_int2(ent_pos[q.x], ent_pos[q.y]);  // Y records are camera-major
}
void su_pair_gather(hipStream_t s, int n, const int* idx, const int2* ef, const int* ent_pos, int2* pairs) {
  if (n > 0) k_su_pair_gather<<<su_grid(n), kSuBlock, 0, s>>>(n, idx, ef, ent_pos, pairs);
}

// ---- (19) explicit-S block tiles (build_schur_tiles, small camera sets) ----
// per point: its entries as (slot, camera) sorted by (camera, slot); distinct cameras m[p]
__global__ void k_su_tile_sort(int NP, const int* __restrict__ ptr, const int* __restrict__ cam,
                               const int* __restrict__ os, int2* __restrict__ sch, int* __restrict__ m) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= NP) return;
  const int b = ptr[p], e = ptr[p + 1];
  for (int i = b; i < e; ++i) {  // insertion sort in place (short lists; keys are unique)
    const int2 v = make_int2(os[i], cam[i]);
    int j = i;
    while (j > b) {
      const int2 u = sch[j - 1];
      if (u.y < v.y || (u.y == v.y && u.x < v.x)) break;
      sch[j] = u;
      --j;
    }
    sch[j] = v;
  }
  int c = 0;
  for (int i = b; i < e; ++i) c += (i == b || sch[i].y != sch[i - 1].y);
  m[p] = c;
}
void su_tile_sort(hipStream_t s, int NP, const int* pt_ent_ptr, const int* ent_cam, const int* ent_os, int2* sch,
                  int* m) {
  if (NP > 0) k_su_tile_sort<<<su_grid(NP), kSuBlock, 0, s>>>(NP, pt_ent_ptr, ent_cam, ent_os, sch, m);
}
// one 64-thread block per batch, thread = point of the batch: the header (mask per camera,
// records before each camera) and the records ordered (camera, point) inside the batch
__global__ __launch_bounds__(64) void k_su_tile_batch(int NC, const int* __restrict__ batch_pt,
                                                      const int* __restrict__ batch_rec, const int* __restrict__ ptr,
                                                      const int2* __restrict__ sch, const int4* __restrict__ obs_idx,
                                                      int hdr_bytes, unsigned char* __restrict__ hdr,
                                                      int4* __restrict__ rec, int4* __restrict__ robs) {
  extern __shared__ unsigned long long tb_lds[];
  unsigned long long* mask = tb_lds;                       // [NC]
  int* off = reinterpret_cast<int*>(tb_lds + NC);          // [NC + 1]
  const int b = blockIdx.x, t = threadIdx.x;
  for (int c = t; c < NC; c += 64) mask[c] = 0ull;
  for (int c = t; c <= NC; c += 64) off[c] = 0;
  __syncthreads();
  const int p = batch_pt[b] + t;
  const bool live = p < batch_pt[b + 1];
  if (live)
    for (int i = ptr[p]; i < ptr[p + 1]; ++i)
      if (i == ptr[p] || sch[i].y != sch[i - 1].y) {
        __hip_atomic_fetch_or(mask + sch[i].y, 1ull << t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(off + sch[i].y + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
  __syncthreads();
  if (t == 0)
    for (int c = 0; c < NC; ++c) off[c + 1] += off[c];
  __syncthreads();
  unsigned long long* hm = reinterpret_cast<unsigned long long*>(hdr + (size_t)b * hdr_bytes);
  int* ho = reinterpret_cast<int*>(hdr + (size_t)b * hdr_bytes + 8 * (size_t)NC);
  for (int c = t; c < NC; c += 64) hm[c] = mask[c];
  for (int c = t; c <= NC; c += 64) ho[c] = off[c];
  if (!live) return;
  const unsigned long long below = (1ull << t) - 1ull;
  int r = -1;
  for (int i = ptr[p]; i < ptr[p + 1]; ++i) {
    const int c = sch[i].y;
    if (i > ptr[p] && c == sch[i - 1].y) {
      rec[r].y++;
      continue;
    }
    r = batch_rec[b] + off[c] + __popcll(mask[c] & below);
    rec[r] = make_int4(i, 1, p, c);
    const int4 oi = obs_idx[sch[i].x >> 1];  // the slot's observation: (point, ext0, ext1, intr)
    robs[r] = make_int4(sch[i].x, oi.y, oi.z, oi.w);
  }
}
void su_tile_batch(hipStream_t s, int nbatch, int NC, const int* batch_pt, const int* batch_rec, const int* pt_ent_ptr,
                   const int2* sch, const int4* obs_idx, int hdr_bytes, unsigned char* hdr, int4* rec, int4* robs) {
  if (nbatch <= 0) return;
  const size_t lds = sizeof(unsigned long long) * (size_t)NC + sizeof(int) * ((size_t)NC + 1);
  k_su_tile_batch<<<nbatch, 64, lds, s>>>(NC, batch_pt, batch_rec, pt_ent_ptr, sch, obs_idx, hdr_bytes, hdr, rec,
                                          robs);
}
// block hit counts from every 4th point: the points that see both cameras of the block
// (integer counts: the order of the adds does not matter)
__global__ __launch_bounds__(kSuBlock) void k_su_tile_hits(int NP, int nb, const int* __restrict__ ptr,
                                                           const int2* __restrict__ sch, int* __restrict__ hits) {
  extern __shared__ int th_lds[];  // [nb]
  for (int k = threadIdx.x; k < nb; k += blockDim.x) th_lds[k] = 0;
  __syncthreads();
  const int p = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (p < NP) {
    const int b = ptr[p], e = ptr[p + 1];
    for (int x = b; x < e; ++x) {
      if (x > b && sch[x].y == sch[x - 1].y) continue;
      const int cx = sch[x].y;
      const int base = (cx * (cx + 1)) >> 1;
      for (int y = b; y <= x; ++y) {
        if (y > b && sch[y].y == sch[y - 1].y) continue;
        atomicAdd(th_lds + base + sch[y].y, 1);
      }
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < nb; k += blockDim.x)
    if (th_lds[k]) atomicAdd(hits + k, th_lds[k]);
}
void su_tile_hits(hipStream_t s, int NP, int nb, const int* pt_ent_ptr, const int2* sch, int* hits) {
  const long long ns = (NP + 3) / 4;
  if (ns > 0) k_su_tile_hits<<<su_grid(ns), kSuBlock, sizeof(int) * (size_t)nb, s>>>(NP, nb, pt_ent_ptr, sch, hits);
}

}  // namespace dab
