// dab_wave.h — wave64 reductions and segmented scans on DPP lane moves (gfx9 DPP
// controls: quad_perm, row_shr, row_bcast:15/31). These replace ds_bpermute-based
// shuffles in every reduction of the hot path: a DPP move is a VALU modifier, a shuffle
// is an LDS round trip. All orders are fixed, so results are bitwise reproducible.
#pragma once
#include <hip/hip_runtime.h>

#include <climits>

namespace dab {

// value of lane (i - shift pattern) per DPP control; lanes without a source keep `old`
template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf>
__device__ __forceinline__ double dpp_f64(double v, double old) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), CTRL, ROW_MASK, BANK_MASK,
                                             false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), CTRL, ROW_MASK, BANK_MASK,
                                             false);
  return __hiloint2double(hi, lo);
}
template <int CTRL, int ROW_MASK = 0xf, int BANK_MASK = 0xf>
__device__ __forceinline__ int dpp_i32(int v, int old) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, ROW_MASK, BANK_MASK, false);
}

// Sum over the 64 lanes; the total is in lane 63 (other lanes hold partials). Inside a
// row every source lane exists (xor 1, xor 2, half-row mirror, row mirror), so those
// moves need no `old` operand; only the two row broadcasts are masked.
template <int CTRL>
__device__ __forceinline__ double dpp_full_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_sum_lane63(double v) {
  v += dpp_full_f64<0xb1>(v);        // quad_perm [1,0,3,2]
  v += dpp_full_f64<0x4e>(v);        // quad_perm [2,3,0,1]
  v += dpp_full_f64<0x141>(v);       // row_half_mirror
  v += dpp_full_f64<0x140>(v);       // row_mirror: every lane holds its row sum
  v += dpp_f64<0x142, 0xa>(v, 0.0);  // row_bcast:15 -> rows 1, 3
  v += dpp_f64<0x143, 0xc>(v, 0.0);  // row_bcast:31 -> rows 2, 3
  return v;
}

// Fixed-order sums over the 64 lanes of K <= 32 values at once, by transposition: a
// v_permlane32_swap of two values leaves value a's lane-pair sums in lanes 0-31 and b's
// in lanes 32-63 after one add (3 instructions per two values), a v_permlane16_swap does
// the same inside each half, and a 16-lane row sum finishes four values per register.
// ~6 VALU per value against ~18 for a full-wave DPP sum of each value. The total of value
// k lands in out[k], stored by one lane (lane 16 g + 15 of register j, k = 4 j + {0,2,1,3}[g]).
__device__ __forceinline__ double swap32_add(double a, double b) {
  const auto l = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(a), (unsigned)__double2loint(b), false, false);
  const auto h = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(a), (unsigned)__double2hiint(b), false, false);
  return __hiloint2double((int)h[0], (int)l[0]) + __hiloint2double((int)h[1], (int)l[1]);
}
__device__ __forceinline__ double swap16_add(double a, double b) {
  const auto l = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(a), (unsigned)__double2loint(b), false, false);
  const auto h = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(a), (unsigned)__double2hiint(b), false, false);
  return __hiloint2double((int)h[0], (int)l[0]) + __hiloint2double((int)h[1], (int)l[1]);
}
template <int K>
__device__ __forceinline__ void wave_sums_transposed(const double (&v)[K], double* out) {
  static_assert(K <= 32, "at most 32 values");
  constexpr int N1 = (K + 1) / 2, N2 = (N1 + 1) / 2;
  double r1[2 * N2];
#pragma unroll
  for (int i = 0; i < N1; ++i) r1[i] = swap32_add(v[2 * i], 2 * i + 1 < K ? v[2 * i + 1] : 0.0);
  if constexpr (N1 < 2 * N2) r1[N1] = 0.0;
  const int lane = threadIdx.x & 63, grp = lane >> 4;
  const int kofs = (grp == 1) ? 2 : (grp == 2) ? 1 : grp;  // {0, 2, 1, 3}
#pragma unroll
  for (int j = 0; j < N2; ++j) {
    double t = swap16_add(r1[2 * j], r1[2 * j + 1]);
    t += dpp_full_f64<0xb1>(t);   // quad_perm [1,0,3,2]
    t += dpp_full_f64<0x4e>(t);   // quad_perm [2,3,0,1]
    t += dpp_full_f64<0x141>(t);  // row_half_mirror
    t += dpp_full_f64<0x140>(t);  // row_mirror: every lane holds its 16-lane sum
    const int k = 4 * j + kofs;
    if ((lane & 15) == 15 && k < K) out[k] = t;
  }
}

// Y records are planar: element j of record i at Y[j * stride + i], so every pass over
// them (one lane per record) issues fully coalesced loads and stores.
template <class YT>
__device__ __forceinline__ void load_yplane(const YT* __restrict__ Y, size_t stride, size_t i, double (&y)[18]) {
#pragma unroll
  for (int j = 0; j < 18; ++j) y[j] = (double)Y[j * stride + i];
}
template <class YT>
__device__ __forceinline__ void store_yplane(YT* __restrict__ Y, size_t stride, size_t i, const double (&y)[18]) {
#pragma unroll
  for (int j = 0; j < 18; ++j) Y[j * stride + i] = (YT)y[j];
}

}  // namespace dab
