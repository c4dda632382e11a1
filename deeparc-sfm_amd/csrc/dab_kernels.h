// dab_kernels.h — launchers of the gfx950 kernels (dab_kernels.hip, dab_chol.hip).
#pragma once
#include <string>
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dab {

constexpr int kCamTab = 32;   // doubles per extrinsic table: R(9) t(3) Rd(9) Jd(9) pad(2)
constexpr int kIntr = 8;      // doubles per intrinsic: cx cy fx fy k0 k1 0 0
constexpr int kYRec = 18;     // elements per Y_e record (6x3), fp64 or fp32 (pcg_fp32)

// Y records of one LM step, planar (element j of record i at j * stride + i), in two
// layouts: cm[18][NE] by camera-major position (camera-side passes) and pm[2][18][NS] by
// observation slot, one record set per extrinsic slot of the observation (point-side
// passes walk the SELL slots with lane = point). fp64, or fp32 for pcg_fp32.
struct YBufs {
  void* cm;
  void* pm;
  bool f32;
};
constexpr int kRedBlock = 256;
// fixed-point cost accumulators (cost_fx_commit): kFxCopies shards of 128 B. A work-group's
// partial sum of r^2 is split into kFxLimbs integer limbs of 50 bits each, limb k in units
// of 2^(50 * (2 - k)) (2^100, 2^50, 1, 2^-50, 2^-100), so any finite partial below 2^150
// is held exactly down to 2^-100; word kFxBad counts non-finite partials. Integer adds are
// associative: the total is the same in any arrival order and across ranks, and no word
// can wrap (each limb < 2^50 + 1, at most 2^11 adds per word over every rank).
constexpr int kFxStride = 16;   // 8-B words per shard
constexpr int kFxCopies = 32;   // shards (work-group b adds into shard b % kFxCopies)
constexpr int kFxWords = kFxStride * kFxCopies;
constexpr int kFxLimbs = 5;
constexpr int kFxBad = kFxLimbs;  // word of the non-finite count
// word kFxErr of shard 0: error bits of the pass that filled the set (k_eval_bal's bounded
// waits). It is zeroed with the set and summed by the cost's all-reduce, so a wait that ran
// out on one rank is seen by every rank at the same read.
constexpr int kFxErr = kFxBad + 1;
inline unsigned long long cost_fx_err(const unsigned long long* words) { return words[kFxErr]; }
// host side: the summed shards of one set -> {sum r^2, non-finite count}
inline void cost_fx_total(const unsigned long long* words, double& sum, double& bad) {
  unsigned long long acc[kFxLimbs + 1] = {0, 0, 0, 0, 0, 0};
  for (int c = 0; c < kFxCopies; ++c)
    for (int i = 0; i <= kFxLimbs; ++i) acc[i] += words[kFxStride * c + i];
  const double unit[kFxLimbs] = {0x1p100, 0x1p50, 1.0, 0x1p-50, 0x1p-100};
  sum = 0.0;
  for (int i = 0; i < kFxLimbs; ++i) sum += (double)acc[i] * unit[i];  // largest limb first
  bad = (double)acc[kFxBad];
}
constexpr int kChunk = 4096;  // max entries per reduction chunk (C3: one chunk per camera)
// max records per pair-major chunk (k_eval_pair; pairs are cut into equal pieces). C5
// (945 pairs of 9.5-10 K records), k_eval_pair per piece count: 5 pieces 200 us, 4 pieces
// 149-151, 3 pieces 190, 2 pieces 154-156 (the launch runs in rounds of two work-groups per
// CU; the 4-piece cut fills its last round best)
constexpr int kPairChunk = 2560;
constexpr int kSlotBit = 1 << 30;  // cm_idx.w flag: the entry is the ring (slot 1) camera

// Device-side problem view. Observations are point-major ("s" order). An "entry" is an
// observation slot whose extrinsic is free; entries have a point-major index e and a
// camera-major position pos (Y records live at pos). cm_idx / cm_xy are a static
// camera-major copy of the observation inputs, so camera-side passes stream them.
struct DevView {
  int N;          // observation slots (SELL-64 layout, padding slots have point -1)
  int NP;         // points (local, referenced)
  int E;          // extrinsics
  int NC;         // free cameras
  int NE;         // entries
  int NI;         // intrinsics
  int nslice;     // SELL-64 slices (64 points each)
  int any_comp;   // some observation is arc∘ring (ext1 >= 0)
  int uni_affine;  // chunk_uni[c] == (c + uni_ox, c + uni_oi) for every camera chunk c (one
  int uni_ox, uni_oi;  // chunk per free camera): k_eval_bal's frames skip that load
  const int4* obs_idx;      // (point, ext0, ext1, intr)
  const double2* obs_xy;
  const int4* cm_idx;       // [NE] obs_idx of the entry's observation, w |= kSlotBit for slot 1
  const double2* cm_xy;     // [NE]
  const int* slice_off;     // [nslice+1] first slot of each slice (slice length = 64 x longest track)
  const int* pt_ent_ptr;    // [NP+1]
  const int* ent_os;        // [NE] s*2+slot (point-major)
  const int* ent_cam;       // [NE]
  const int* ent_pt;        // [NE]
  const int* ent_pos;       // [NE] camera-major position
  const int* cm_pt;         // [NE] point of the entry at camera-major position
  const int* ext_col;       // [E] free camera index or -1
  const double* intr;       // [NI][kIntr]
  const int2* chunk_uni;    // [nchunk] (ext, intr) shared by every entry of the chunk, or (-1, -1)
  const int* obs_e;         // [N] (streamed fused pass; null otherwise) ext0 | intr << 16 of a
                            // single-extrinsic slot, -1 for padding
};

// camera-side chunks split by whether one camera/intrinsic serves the whole chunk
struct ChunkLists {
  int nchunk = 0, nuni = 0, ngen = 0;
  const int* uni = nullptr;  // [nuni] chunk ids with chunk_uni >= 0
  const int* gen = nullptr;  // [ngen] the others
};

// camera tables for all extrinsics from ext[E][6]
void launch_cam_tables(hipStream_t s, int E, const double* ext, double* camtab);
// Point side of the evaluation pass (rows a1-a4, matrix-free): residual + d r / d X per
// observation reduced into V[6][NP], g[3][NP] (one SELL slice per block, lane = point;
// wps = 4 | 8 | 16 waves per slice reading camtab; 0 / -2 = 4 / 2 waves per slice with R,t
// built from ext into LDS on a persistent grid), cost[2] = {sum r^2, non-finite count}
// (partial[grid][2] is scratch; arrivals is a zeroed counter the kernel leaves zeroed).
// wps <= -100 (the prefetch kernels) add the cost into the fixed-point shards costfx
// [kFxWords] (zeroed by the previous pass) and zero fx_next [kFxWords] for the next pass;
// the other variants write cost[2].
void launch_eval_points(hipStream_t s, const DevView& v, const double* points, const double* ext,
                        const double* camtab, double* V, double* g, double* partial, unsigned* arrivals,
                        double* cost, unsigned long long* costfx, unsigned long long* fx_next, int grid, int wps);
inline bool eval_points_fx(int wps) { return wps <= -100 && (-wps - 100) / 1000 != 64; }
// whether the chosen variant reads camtab (the LDS variants build R,t from ext themselves)
bool eval_points_needs_camtab(int wps);
bool eval_points_lds_fits(int E);
// Full Jacobian planes (parity API): Jfull[30][N], r[N]
void launch_jacobian_full(hipStream_t s, const DevView& v, const double* points,
                          const double* camtab, double* r, double* Jfull);
// residual only, with per-block partial sums of r^2 and a non-finite count
void launch_residual(hipStream_t s, const DevView& v, const double* points, const double* camtab,
                     double* r_out /*nullable*/, double* partial /*[grid][2]*/, int grid);
// filterPoint3d masks (DeepArcManager.cc:332-424): slot_keep[N slots], pt_keep[NP]
void launch_filter(hipStream_t s, const DevView& v, const double* points, const double* camtab, double eb,
                   const double c[3], double radius, unsigned char* slot_keep, unsigned char* pt_keep);
// camera side of the evaluation pass (matrix-free, camera-major inputs):
//  U/g: per entry 21 (Jc^T Jc upper) + 6 (Jc^T r) -> partial[chunk][27]
void launch_eval_cams(hipStream_t s, const DevView& v, const ChunkLists& cl, const int* chunk_beg,
                      const double* points, const double* ext, const double* camtab, double* partial);
// Fused evaluation pass for BAL-shaped problems (camera side -> ug[NC][27] directly,
// point side -> V, g, cost in fixed point as launch_eval_points): one launch, camera and
// point waves side by side. fused_eval_fits: whether the problem qualifies for `grid`.
bool fused_eval_fits(const DevView& v, int nchunk, int ngen, int ncross, int grid);
// k_eval_bal (needs v.obs_e, the packed point-side records): side kSideBoth both halves;
// kSidePoints the point side only (V, g, cost; the camera waves return at once, no frames);
// kSideCams the camera side only (ug; the point waves return at once, no tables, no
// intrinsic DMA) — the multi-rank split schedule runs the same machine code with a run-time
// side, so both schedules give bitwise the same sums; | kSideTestTimeout (a test flag) a frame
// wait that never completes, so the pass must fail closed. Builds with -DDAB_ABLATIONS add the
// timing ablations 3..6 (wrong results); release builds never launch them (eval_pass
// refuses DAB_EVAL_SIDE outside {0, 7}). camtab non-null: R,t and the camera frames copied
// from the tables of the current x instead of built. err: sticky per-handle error word;
// costfx[kFxErr] (shard 0) gets the same bits, so the error travels with the cost's
// all-reduce and every rank fails the same call (0 = ok)
constexpr int kSideBoth = 0, kSidePoints = 1, kSideCams = 2, kSideTestTimeout = 16;
void launch_eval_bal(hipStream_t s, const DevView& v, const int* chunk_beg, const double* points, const double* ext,
                     const double* camtab, double* V, double* g, double* ug, unsigned long long* costfx,
                     unsigned long long* fx_next, unsigned* err, int grid, int side);
//  arc∘ring cross blocks Jc0^T Jc1 over composed observations (pair-major copy) -> partial[chunk][36]
void launch_eval_cross(hipStream_t s, const DevView& v, int nchunk, const int* chunk_beg, const int4* x_idx,
                       const double2* x_xy, const double* points, const double* camtab, double* partial);
// The rig's composed observations with both cameras free, one pair-major pass: per chunk
// the cross block -> xpart[chunk][36] and both cameras' [U | g] -> cpart[chunk][54]
// (arc 27 | ring 27); k_cam_final adds those halves to the camera-major partials of the
// other entries (launch_eval_cams_gen over their own chunks).
bool pair_eval_fits(int E, int NI);  // the tables fit LDS (small_tabs_fit)
void launch_eval_pair(hipStream_t s, const DevView& v, int nchunk, const int* chunk_beg, const int4* x_idx,
                      const double2* x_xy, const double* points, const double* camtab, double* xpart,
                      double* cpart, bool uni_intr);
void launch_cam_final(hipStream_t s, int NC, const int* seg_chunk, const double* partial, const int* xcam_ptr,
                      const int* xcam_list, const double* cpart, double* ug);
void launch_eval_cams_gen(hipStream_t s, const DevView& v, int nchunk, const int* chunk_beg, const double* points,
                          const double* ext, const double* camtab, double* partial);
//  final: seg_out[seg][K] = sum of partial chunks [seg_chunk[seg], seg_chunk[seg+1])
//  (max_chunks = the largest number of chunks of one segment: > 8 uses a block per segment)
void launch_seg_final(hipStream_t s, int nseg, int K, const int* seg_chunk, const double* partial,
                      double* out, int max_chunks = 1);
// generic grid-level sum of partial[grid][K] -> out[K] (single block, fixed order); the
// components whose bit is set in max_mask are combined with max instead of +.
void launch_final_sum(hipStream_t s, int grid, int K, const double* partial, double* out,
                      unsigned max_mask = 0u);
// camera-side norms (one block): out[5] = {sum (ext-ext_c)^2, sum ext_c^2,
//   max |x-(x-g)|, sum (x-(x-g))^2, sum ext^2} over free camera components
void launch_cam_norms(hipStream_t s, int E, const int* ext_col, const double* ext,
                      const double* ext_c, const double* ug, double* out);

// ---- per-iteration (LM step) kernels --------------------------------------------------
struct StepScalars {
  double radius, min_diag, max_diag;
};
// point factor: Vs = s V s + D^2 = L L^T -> PU[NP][6] = diag(s) L^-T (upper: 00 01 02 11
// 12 22), q = L^-1 (s g) -> q[NP][4]
void launch_point_factor(hipStream_t s, const DevView& v, const double* V, const double* g,
                         const double* scale_p, StepScalars sc, double* PU, double* q, int* fail);
// entry Y = (s_c ∘ Jc^T Jp) PU_p (re-evaluated) -> Y.cm (camera-major pass) and Y.pm
// (slot pass; with_pm = false skips it)
// rec (fp64 Y only): the camera-major pass writes [NE][18] records there instead of Y.cm
void launch_entry_y(hipStream_t s, const DevView& v, const double* points, const double* camtab,
                    const double* scale_c, const double* PU, YBufs Y, bool with_pm, double* rec = nullptr);
// S blocks (Y part): packed[blk][36] = - sum_pairs Y_row Y_col^T (pairs hold positions;
// Y = the fp64 camera-major planes, stride NE; Yr = scratch [NE][18] for the records, or
// Y = nullptr when Yr already holds them). S != nullptr (one rank): the blocks go straight
// into the dense lower S at (6 c, 6 d) of blk_cam[blk], and the nzero lower blocks without
// pairs (blk_zero) are zeroed, instead of packed[] and launch_s_unpack's zero + scatter
void launch_s_blocks(hipStream_t s, int nblk, const int* blk_pair_beg, const int2* pairs,
                     const double* Y, int NE, double* packed, double* Yr, double* S = nullptr, int lds = 0,
                     const int2* blk_cam = nullptr, int nzero = 0, const int2* blk_zero = nullptr);
// Explicit S for small camera sets without pair tables (k_schur_y + k_schur_tiles): every
// thread of a work-group owns one 6x6 block of the lower block triangle of S (numbered
// row-major: block (c, d <= c) = c (c+1)/2 + d) and sums it in registers over the records of
// its group of points; fp64, one fixed order per block. The rhs part is summed in fixed point:
// row 6 c + r in units of 2^(kx[R] + kq - 60).
constexpr int kMfCamsMax = 160;  // small camera sets (matrix-free PCG, explicit S tiles)
constexpr int kTileMaxRec = 32;  // distinct free cameras per point (tile path limit)
__host__ __device__ inline long long tri_n(long long i) { return (i * (i + 1)) >> 1; }
struct SchurTiles {
  int ntile, ngroup, nbatch, nelem;  // nelem = 36 NC (NC + 1) / 2
  int nrec;                          // records: distinct (point, free camera) pairs
  int kq;                            // rhs exponent: 2^kq >= sqrt(2 cost)
  // records are ordered by (batch, camera, point): inside a batch the records of cameras
  // 0..c form a prefix, and the record of (point pl, camera c) is
  // off[c] + popcount(mask[c] & ((1 << pl) - 1)) from the batch start
  const int* batch_rec;              // [nbatch + 1] first record of each batch (<= batch_cap records)
  const unsigned char* hdr;          // [nbatch][hdr_bytes]: mask[NC] (u64, bit = point of the batch) |
                                     // off[NC + 1] (int, records before camera c in the batch)
  int hdr_bytes;                     // 16-B multiple
  int batch_cap;                     // records per batch (one LDS buffer)
  int single;                        // 1: one LDS buffer of kTileLdsMax (batches twice as large, each
                                     // batch's DMA waited for); 0: two buffers, the next batch in flight
  const int* tile_clast;             // [ntile] last row camera of the tile (its records: a batch prefix)
  const int* tile_slot;              // [ntile][2 kTileThreads] block owned by (thread, half) or -1,
                                     // balanced by the blocks' sampled hit counts
  const int4* rec_info;              // [nrec] (first entry in sch_ent, entry count, point, camera)
  const int4* rec_obs;               // [nrec] the first entry's (observation slot 2 s + camera slot,
                                     // ext0, ext1, intr): k_schur_y streams it instead of two gathers
  const int2* sch_ent;               // [NE] (ent_os, camera), sorted by camera inside each point
  const int* kx;                     // [6 NC] rhs row exponents (launch_schur_scale)
  double* partial;                   // [nslot][stride] per-slot block sums
  size_t stride;                     // nelem
  // load balance: tile t's batches are cut into ngroup * tile_sub[t] slots (a heavy tile
  // gets more work-groups); the launch has ngroup * nsub work-groups, nsub = sum of tile_sub
  int nsub;
  const int* tile_sub;               // [ntile] work-groups per group of batches
  const int* tile_subbeg;            // [ntile + 1] prefix of tile_sub
  const int* blk_nslot;              // [nblocks] slots holding the block's partials (k_schur_sum)
};
constexpr int kTileThreads = 512;     // threads of a k_schur_tiles work-group (two blocks each)
constexpr size_t kTileLdsMax = 163840;            // LDS of one k_schur_tiles work-group (at most)
int schur_tile_batch_cap(int NC, bool single);    // records per batch (one LDS buffer, or one of two)
int schur_tile_hdr_bytes(int NC);                 // batch header bytes (16-B multiple)
void launch_schur_scale(hipStream_t s, int NC, const double* ug, const double* scale_c, int* kx);
// Y of every record -> yrec[nrec][18]; rhs fixed-point sums added into rhs_out[6 NC]
void launch_schur_y(hipStream_t s, const DevView& v, const double* points, const double* camtab, const double* PU,
                    const double* q, const double* scale_c, const SchurTiles& a, double* yrec,
                    unsigned long long* rhs_out);
void launch_schur_tiles(hipStream_t s, const double* yrec, const SchurTiles& a, int NC);
// sblk[i] = sum of the slots' partials of element i in slot order (blk_nslot[i / 36] slots)
void launch_schur_sum_tiles(hipStream_t s, const SchurTiles& a, double* out);
void launch_schur_sum(hipStream_t s, int ngroup, size_t stride, size_t count, const double* partial, double* out);
// S lower rows 0..n-1 = -Schur part, ybc = -rhs part (then launch_s_add_u)
void launch_schur_unpack(hipStream_t s, int NC, const double* sblk, const unsigned long long* rfx, const int* kx,
                         int kq, double* S, int lds, double* ybc);
// adds the U part (+ D^2) and cross blocks, writes the rhs row n = s_c g_c + ybc
void launch_s_add_u(hipStream_t s, int NC, const double* ug, int ncross, const int2* cross_cam, const double* Ucross,
                    const double* scale_c, StepScalars sc, const double* ybc, double* S, int lds);
// camera rhs partial: per position -Y q_p -> partial[chunk][6]
// (Y planes, or rec = true: [NE][18] records)
void launch_cam_rhs_partial(hipStream_t s, const DevView& v, int nchunk, const int* chunk_beg,
                            const double* Y, const double* q, double* partial, bool rec = false);
// dense S (row-major, lower, ld = lds, n = 6 NC, n+1 rows): zero, scatter packed blocks,
// add the U part + D^2, write rhs b = s_c g_c + ybc into row n.
// ug: [NC][27] = (U upper-packed 21 | g_c 6) per camera
void launch_s_unpack(hipStream_t s, int NC, int nblk, const int2* blk_cam, const double* packed,
                     const double* ug, int ncross, const int2* cross_cam,
                     const double* Ucross /*[ncross][36]*/, const double* scale_c, StepScalars sc,
                     const double* ybc /*[NC][6]*/, double* S, int lds);
// delta_p = -PU (q - sum_e Y_e^T y_c) -> dp[3][NP]
void launch_backsub(hipStream_t s, const DevView& v, const double* PU, const double* q, YBufs Y,
                    const double* yc, double* delta_p);
// x_c = x + delta for points; partial[grid][2] = {sum (x-xc)^2, sum xc^2}
void launch_axpy_points(hipStream_t s, int NP, const double* x, const double* d, double* xc,
                        double* partial, int grid);
void launch_cam_candidate(hipStream_t s, int E, const int* ext_col, const double* ext,
                          const double* yc, const double* scale_c, double* ext_c,
                          double* delta_c);
// model cost change + candidate cost in one observation pass:
//  partial[grid][3] = { sum -(m.(r+m/2)), sum rc^2, nonfinite }
void launch_candidate(hipStream_t s, const DevView& v, const double* points, const double* camtab,
                      const double* delta_p, const double* delta_c, const double* camtab_c, double* partial,
                      int grid);
// gradient norms over points: partial[grid][3] = {max |x-(x-g)|, sum (x-(x-g))^2, sum x^2}
void launch_grad_points(hipStream_t s, int NP, const double* x, const double* g /*[3][NP]*/,
                        double* partial, int grid);

// ---- implicit-Schur PCG (dab_pcg.hip) -------------------------------------------------------
enum { kPcgRunning = 0, kPcgSuccess = 1, kPcgNoConvergence = 2, kPcgFailure = 3 };
struct PcgState {
  double rho, Q0, alpha, eta, norm_b, pad[3];  // pad[0]: beta of the multi-work-group update
  int iter, status, min_iter, max_iter;
};
// per chunk: 21 upper of sum_runs Z Z^T (Z = sum of the run's Y; run[i] = length of the
// same-point run starting at position i, 0 inside a run) | 6 of -sum Y q_p -> partial[chunk][27]
void launch_pcg_diag_rhs_partial(hipStream_t s, const DevView& v, int nchunk, const int* chunk_beg,
                                 const int* run, YBufs Y, const double* q, double* partial);
// per camera: Ad = s U s + D^2 [NC][36], Minv = (Ad - sum Y Y^T)^-1 [NC][36],
// b = s g_c - sum Y q, x = 0, r = b; fail[0] |= 1 if a block is not positive definite
void launch_pcg_setup(hipStream_t s, int NC, const double* ug, const double* scale_c, StepScalars sc,
                      const double* red, double* Ad, double* Minv, double* bvec, double* x, double* r,
                      int* fail);
// norm_b, status, and the first direction (z = M^-1 r, rho, p = z; iteration 1)
void launch_pcg_init(hipStream_t s, int NC, const double* bvec, const int* fail, PcgState* st, double eta,
                     int min_iter, int max_iter, const double* Minv, const double* r, double* z, double* p);
// the two Y passes of S vec: t[NP][4], partial[chunk][6] (= -sum Y t per chunk)
// fused single-pass matvec for NC <= 160 cameras: w = -sum_e Y_e t_p(e) with the point-major
// records only; partial[grid][6 NC] scratch
bool pcg_fused_fits(int NC);
int pcg_fused_grid(int NP, int ncu);
void launch_pcg_fused(hipStream_t s, const DevView& v, YBufs Y, const double* vec, double* partial, double* w,
                      int grid, const PcgState* st);
void launch_pcg_matvec_passes(hipStream_t s, const DevView& v, int nchunk, const int* chunk_beg, YBufs Y,
                              const double* vec, double* t, double* partial, const PcgState* st);
// mode 0: q = S p, alpha, x, r, Q-test; 1: q = S p, alpha, x; 2: r = b - S x, Q-test.
// Modes 0 and 2 end with the next direction (z = M^-1 r, rho, beta, p) when still running.
// w[NC][6] = all-reduced Y part of the product; xptr/xlist: per-camera CSR of cross blocks
// (code = 2*k + (camera is c1)), nullable when there are none.
// The same CG update spread over work-groups (three launches, last-arriver grid sums):
// partial[cg_partial_size(NC)] scratch, cnt a zeroed counter (left zeroed).
void launch_cg_update(hipStream_t s, int NC, int mode, const double* Ad, const double* w, const int* xptr,
                      const int* xlist, const int2* xcam, const double* X, const double* scale_c,
                      const double* bvec, double* p, double* q, double* x, double* r, PcgState* st,
                      const double* Minv, double* z, double* partial, unsigned* cnt,
                      const double* wpart = nullptr, int wpart_g = 0);
// wpart: the matrix-free product's [wpart_g][6 NC] work-group partials, summed inside the
// update (one work-group per camera when there are cross blocks) instead of into w first
int cg_partial_size(int NC);
void launch_pcg_update(hipStream_t s, int NC, int mode, const double* Ad, const double* w, const int* xptr,
                       const int* xlist, const int2* xcam, const double* X, const double* scale_c,
                       const double* bvec, double* p, double* q, double* x, double* r, PcgState* st,
                       const double* Minv, double* z);

// ---- matrix-free implicit Schur (small camera sets; dab_kernels.hip) -------------------
// Y_e is never stored: rows are re-evaluated per pass (tables and s_c staged in LDS).
bool mf_schur_fits(int NC, int E, int NI);
int mf_grid(int NP, int ncu);
// Y part of S vec: partial[grid][6 NC] scratch -> w[NC][6] (fixed order; w = nullptr: the
// partials are left for launch_cg_update's wpart)
void launch_mf_product(hipStream_t s, const DevView& v, const double* points, const double* camtab,
                       const double* scale_c, const double* PU, const double* vec, double* partial, double* w,
                       int grid, const PcgState* st);
// the same product with fp32 per-observation arithmetic and fp64 sums (mixed precision)
void launch_mf_product32(hipStream_t s, const DevView& v, const double* points, const double* camtab,
                         const double* scale_c, const double* PU, const double* vec, double* partial, double* w,
                         int grid, const PcgState* st);
// dp[3][NP] = -PU (q - sum_e Y_e^T y_c)
void launch_mf_backsub(hipStream_t s, const DevView& v, const double* points, const double* camtab,
                       const double* scale_c, const double* PU, const double* q, const double* yc, double* dp,
                       int grid);
// per chunk: 21 of sum Z Z^T over same-point runs | 6 of -sum Y q -> partial[chunk][27]
// run_beg[nchunk + 1]: each chunk's runs in run_rec {first position, length, point, camera}
void launch_mf_diag_rhs(hipStream_t s, const DevView& v, int nchunk, const int* run_beg, const int4* run_rec,
                        const double* points, const double* camtab, const double* scale_c, const double* PU,
                        const double* q, double* partial);
// fixed-order sum of the per-work-group product partials (dab_pcg.hip)
void launch_pcg_fused_final(hipStream_t s, int grid, int NC6, const double* partial, double* w, const PcgState* st);

// ---- dense Cholesky (dab_chol.hip) -------------------------------------------------------
// Factor the (n+1)x(n+1) augmented lower matrix [S b; b^T *] in place (row-major, ld = lda):
// the first n rows end as L and row n as z = L^-1 b; then solve L^T y = z into y.
// d_flag[0] is set when a pivot is not positive. Returns 0, or <0 on a library error.
struct CholCtx;
// Process-wide caches of the handle's runtime objects (each hipStreamCreate / Destroy took
// ~2 ms, a handle makes three): an idle non-blocking stream of the current device, created
// when the cache has none; stream_give synchronises it and keeps it for the next handle.
// pinned_take / pinned_give do the same for small pinned host blocks (by size).
hipStream_t stream_take(int device);
void stream_give(int device, hipStream_t s);
void* pinned_take(size_t bytes);
void pinned_give(void* p, size_t bytes);
CholCtx* chol_create();
void chol_destroy(CholCtx*);
int chol_factor_solve(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y, int* d_flag);
int chol_prepare(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y, int* d_flag);
int chol_guard_check(CholCtx* c, const char* where, std::string* first);
struct Dev;
Dev* chol_mem(CholCtx* c);  // the Cholesky scratch's allocator (dab_devmem.h)

int grid_for(int n, int block, int cap);

// code-object warm-up, one per translation unit (called at handle creation)
void warm_chol();
void warm_kernels();
void warm_pcg();
void warm_p2p();

}  // namespace dab
