// dab_setup.h — device passes of dab_set_problem (dab_setup.hip). Internal, not ABI.
//
// The observation orderings and reduction tables the solver runs on (SELL-64 slots, the
// entry lists, the camera-major copy and its chunks and runs, the pair-major copy of the
// rig's composed observations) are built on the GPU from the caller's arrays: rocPRIM
// radix sorts (stable, so every order is the host counting sort's), scans and
// gather / scatter passes. The results are bitwise those of the host passes in
// dab_solver.hip (kept as the reference path, DAB_SETUP_HOST=1).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace dab {

// rocPRIM wrappers: tmp == nullptr queries *tmp_bytes. 0 on success.
int su_sort_pairs(void* tmp, size_t* tmp_bytes, const int* kin, int* kout, const int* vin, int* vout, int n,
                  int end_bit, hipStream_t s);
int su_exclusive_scan(void* tmp, size_t* tmp_bytes, const int* in, int* out, int n, hipStream_t s);
int su_max(void* tmp, size_t* tmp_bytes, const int* in, int* out, int n, hipStream_t s);
// stable compaction of idx (int4) and xy (double2) by flags (nonzero = keep); *count out
int su_select_flagged_i(void* tmp, size_t* tmp_bytes, const int* in, const unsigned char* flags, int* out,
                        int* count, int n, hipStream_t s);
// runs of equal keys: unique keys, run lengths, number of runs
int su_rle(void* tmp, size_t* tmp_bytes, const int* in, int* unique, int* counts, int* nruns, int n, hipStream_t s);

// (1) point counts, referenced extrinsics, composed flag, index validation.
// flags bit 0: an out-of-range index (the host path's validate() error), bit 1: composed
void su_count(hipStream_t s, int N, const int* obs_point, const int* obs_ext0, const int* obs_ext1,
              const int* obs_intr, int num_points, int num_ext, int num_intr, int* pcount, int* eref, int* flags);
// (2) keys of the device point order (count descending, stable by id; unreferenced last)
void su_point_keys(hipStream_t s, int num_points, const int* pcount, const int* maxcount, int* keys, int* vals,
                   int* nref);
// (3) pt_local[pt_of[l]] = l; lcount[l] = count of local point l
void su_point_local(hipStream_t s, int NP, const int* pt_of, const int* pcount, int* pt_local, int* lcount);
// (4) observation keys: local point of each observation (values = observation ids)
void su_obs_keys(hipStream_t s, int N, const int* obs_point, const int* pt_local, int* keys, int* vals);
// (5) slice lengths: 64 x the longest track of each slice (its first point's)
void su_slice_len(hipStream_t s, int nslice, int NP, const int* lcount, int* slen);
// (6) SELL-64 slots: obs_idx / obs_xy / perm per slot (padding: point -1), free-camera slots
// per point (ne[NP])
void su_slots(hipStream_t s, int NP, int nslice, const int* slice_off, const int* cnt, const int* lcount,
              const int* by_pt, const int* obs_ext0, const int* obs_ext1, const int* obs_intr, const double* obs_xy,
              const int* ext_col, int4* obs_idx, double2* obs_xy_out, int* perm, int* ne);
// (7) entries (free-camera slots), point-major
void su_entries(hipStream_t s, int NP, const int* slice_off, const int* lcount, const int4* obs_idx,
                const int* ext_col, const int* pt_ent_ptr, int* ent_os, int* ent_cam, int* ent_pt);
// (8) first position of every camera in the camera-sorted keys (cam_cnt[NC + 1])
void su_bounds(hipStream_t s, int n, const int* sorted_keys, int nkeys, int* start);
// (9) camera-major copies: ent_pos, cm_pt, cm_idx, cm_xy
void su_camera_major(hipStream_t s, int NE, const int* cam_ent, const int* ent_pt, const int* ent_os,
                     const int4* obs_idx, const double2* obs_xy, int* ent_pos, int* cm_pt, int4* cm_idx,
                     double2* cm_xy);
// (10) runs of one point inside one camera's positions: run length at a run's first
// position, 0 elsewhere (pos_cam: the camera of every position)
void su_runs(hipStream_t s, int NE, const int* pos_cam, const int* cm_pt, int* run);
// (11) per chunk: number of runs (run_cnt), then their records {position, length, point,
// camera} in position order; chunk_uni (the chunk's one (ext, intr), or (-1, -1))
void su_chunk_runs(hipStream_t s, int nchunk, const int* chunk_beg, const int* run, int* run_cnt);
void su_chunk_run_rec(hipStream_t s, int nchunk, const int* chunk_beg, const int* run, const int* cm_pt,
                      const int* pos_cam, const int* run_beg, int4* run_rec);
void su_chunk_uni(hipStream_t s, int nchunk, const int* chunk_beg, const int4* cm_idx, int slot_bit, int2* chunk_uni);
// (12) composed slots with both cameras free: key c0 NC + c1 (or a sentinel), value = slot;
// nvalid counts the keyed slots
void su_cross_keys(hipStream_t s, int NS, const int4* obs_idx, const int* ext_col, int NC, int* keys, int* vals,
                   int* nvalid);
// (13) pair-major copy of the composed slots in sorted order; the points they touch
void su_cross_copy(hipStream_t s, int n, const int* slots, const int4* obs_idx, const double2* obs_xy,
                   int4* x_idx, double2* x_xy, unsigned char* touched);
// (14) count of set bytes
void su_count_flags(hipStream_t s, int n, const unsigned char* flags, int* count);
// neighbouring pair-major records of one (arc, ring) pair with different intrinsics, added to *count
void su_pair_intr(hipStream_t s, int n, const int4* x_idx, int* count);
// (15) entries not paired (camera-major flags) and the stable copy of their records
void su_unpaired_flags(hipStream_t s, int NE, const int4* cm_idx, const int* ext_col, unsigned char* flags,
                       int* flags_i);
void su_gather_cm(hipStream_t s, int n, const int* sel, const int4* cm_idx, const double2* cm_xy, int4* out_idx,
                  double2* out_xy);
// (16) packed point-side records (ext | intr << 16; -1 padding) and the device-order points
void su_obs_e(hipStream_t s, int NS, const int4* obs_idx, int* obs_e);
void su_points(hipStream_t s, int NP, const int* pt_of, const double* raw_points, double* points);
// (17) iota; out[c] = in[idx[c]] (small tables read back to the host)
void su_iota(hipStream_t s, int n, int* out);
void su_gather_at(hipStream_t s, int n, const int* idx, const int* in, int* out);
// (18) explicit-Schur pair tables: per point the count of ordered entry pairs (e, f) with
// cam(e) >= cam(f) (and their 64-bit total, added into *total); the pairs in (point, e, f)
// order as key cam(e) NC + cam(f), value = position, ef = (e, f); after the stable sort by
// key, pairs[i] = (ent_pos[e], ent_pos[f]) of the i-th sorted position
void su_pair_count(hipStream_t s, int NP, const int* pt_ent_ptr, const int* ent_cam, int* cnt,
                   unsigned long long* total);
void su_pair_gen(hipStream_t s, int NP, const int* pt_ent_ptr, const int* ent_cam, const int* poff, int NC, int* keys,
                 int* vals, int2* ef);
void su_pair_gather(hipStream_t s, int n, const int* idx, const int2* ef, const int* ent_pos, int2* pairs);
// (19) explicit-S block tiles: per point its entries as (slot, camera) sorted by (camera,
// slot) and its count of distinct cameras; per batch (64-thread block) the header and the
// records ordered (camera, point); sampled block hit counts (every 4th point, added into
// hits[nb])
void su_tile_sort(hipStream_t s, int NP, const int* pt_ent_ptr, const int* ent_cam, const int* ent_os, int2* sch,
                  int* m);
void su_tile_batch(hipStream_t s, int nbatch, int NC, const int* batch_pt, const int* batch_rec, const int* pt_ent_ptr,
                   const int2* sch, const int4* obs_idx, int hdr_bytes, unsigned char* hdr, int4* rec, int4* robs);
void su_tile_hits(hipStream_t s, int NP, int nb, const int* pt_ent_ptr, const int2* sch, int* hits);
// code-object warm-up (handle creation)
void warm_setup();

}  // namespace dab
