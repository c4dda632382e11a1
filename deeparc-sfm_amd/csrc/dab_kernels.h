// dab_kernels.h — launchers of the gfx950 kernels (dab_kernels.hip, dab_chol.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dab {

constexpr int kCamTab = 32;   // doubles per extrinsic table: R(9) t(3) Rd(9) Jd(9) pad(2)
constexpr int kIntr = 8;      // doubles per intrinsic: cx cy fx fy k0 k1 0 0
constexpr int kRedBlock = 256;
constexpr int kChunk = 1024;  // max elements per reduction chunk

// All pointers are device pointers. Observation arrays are in point-major order.
struct DevView {
  int N;          // observations
  int NP;         // points (local, referenced)
  int E;          // extrinsics
  int NC;         // free cameras
  int NE;         // entries (observation slots whose extrinsic is free)
  int nplanes;    // Jacobian planes (18 or 30)
  const int4* obs_idx;      // (point, ext0, ext1, intr)
  const double2* obs_xy;
  const int* pt_obs_ptr;    // [NP+1]
  const int* pt_ent_ptr;    // [NP+1]
  const int* ent_os;        // [NE] s*2+slot
  const int* ent_cam;       // [NE]
  const int* ent_pt;        // [NE]
  const int* ext_col;       // [E] free camera index or -1
  const double* intr;       // [NI][kIntr]
};

// camera tables for all extrinsics from ext[E][6]
void launch_cam_tables(hipStream_t s, int E, const double* ext, double* camtab);
// residual + Jacobian: r[N] (double2), J[plane][N]
void launch_jacobian(hipStream_t s, const DevView& v, const double* points, const double* camtab,
                     double* r, double* J);
// residual only, with per-block partial sums of r^2 and a non-finite count
void launch_residual(hipStream_t s, const DevView& v, const double* points, const double* camtab,
                     double* r_out /*nullable*/, double* partial /*[grid][2]*/, int grid);
// per-point V (6 unique, unscaled) and g (3) : V[6][NP], g[3][NP]
void launch_point_vg(hipStream_t s, const DevView& v, const double* r, const double* J, double* V,
                     double* g);
// chunked camera-major reductions
//  U/g: per entry 21 (Jc^T Jc upper) + 6 (Jc^T r) -> partial[chunk][27]
void launch_cam_ug_partial(hipStream_t s, const DevView& v, int nchunk, const int* chunk_beg,
                           const int* cam_ent, const double* r, const double* J, double* partial);
//  cross blocks Jc0^T Jc1 over composed observations -> partial[chunk][36]
void launch_cross_partial(hipStream_t s, const DevView& v, int nchunk, const int* chunk_beg,
                          const int* xobs, const double* J, double* partial);
//  final: seg_out[seg][K] = sum of partial chunks [seg_chunk[seg], seg_chunk[seg+1])
void launch_seg_final(hipStream_t s, int nseg, int K, const int* seg_chunk, const double* partial,
                      double* out);
// generic grid-level sum of partial[grid][K] -> out[K] (single block, fixed order); the
// components whose bit is set in max_mask are combined with max instead of +.
void launch_final_sum(hipStream_t s, int grid, int K, const double* partial, double* out,
                      unsigned max_mask = 0u);
// sum of r^2 and non-finite count over r[N] (double2) -> partial[grid][2]
void launch_r_sumsq(hipStream_t s, int N, const double* r, double* partial, int grid);
// camera-side norms (one block): out[5] = {sum (ext-ext_c)^2, sum ext_c^2,
//   max |x-(x-g)|, sum (x-(x-g))^2, sum ext^2} over free camera components; ug as below
void launch_cam_norms(hipStream_t s, int E, const int* ext_col, const double* ext,
                      const double* ext_c, const double* ug, double* out);

// ---- per-iteration (LM step) kernels --------------------------------------------------
struct StepScalars {  // device-side radius etc. are passed by value
  double radius, min_diag, max_diag;
};
// point factor: Vs = s V s + D^2, L = chol(Vs), q = L^-1 (s g). L[6][NP], q[3][NP],
// Dp[3][NP] (the LM D), fail flag (int) set when not PD.
void launch_point_factor(hipStream_t s, const DevView& v, const double* V, const double* g,
                         const double* scale_p, StepScalars sc, double* L, double* q, int* fail);
// entry Y_e = (s_c ∘ Jc^T Jp ∘ s_p) L^-T -> Y[18][NE]
void launch_entry_y(hipStream_t s, const DevView& v, const double* J, const double* scale_p,
                    const double* scale_c, const double* L, double* Y);
// S blocks (Y part): packed[blk][36] = - sum_pairs Y_row Y_col^T
void launch_s_blocks(hipStream_t s, const DevView& v, int nblk, const int* blk_pair_beg,
                     const int2* pairs, const double* Y, double* packed);
// camera rhs partial: per entry -Y_e q_p -> partial[chunk][6]
void launch_cam_rhs_partial(hipStream_t s, const DevView& v, int nchunk, const int* chunk_beg,
                            const int* cam_ent, const double* Y, const double* q, double* partial);
// dense S (row-major, lower, ld = ns, ns = 6 NC): zero, scatter packed blocks, add U part + D^2.
// Also writes rhs b = s_c g_c + ybc into the augmented row ns (S has ns+1 rows).
// ug: [NC][27] = (U upper-packed 21 | g_c 6) per camera
void launch_s_unpack(hipStream_t s, int NC, int nblk, const int2* blk_cam, const double* packed,
                     const double* ug, int ncross, const int2* cross_cam,
                     const double* Ucross /*[ncross][36]*/, const double* scale_c, StepScalars sc,
                     const double* ybc /*[NC][6]*/, double* S, int lds);
// camera LM diagonal only (freeze / no camera): nothing. Point back-substitution:
// y_p = L^-T (q - sum_e Y_e^T y_c); delta_p = -y_p * s_p
void launch_backsub(hipStream_t s, const DevView& v, const double* L, const double* q,
                    const double* Y, const double* yc, const double* scale_p, double* delta_p);
// x_c = x + delta for points (3 NP) ; cameras: ext_c = ext + delta_c for free cams
void launch_axpy_points(hipStream_t s, int NP, const double* x, const double* d, double* xc,
                        double* partial /*[grid][3]: step^2, x^2(xc), -*/, int grid);
void launch_cam_candidate(hipStream_t s, int E, const int* ext_col, const double* ext,
                          const double* yc, const double* scale_c, double* ext_c,
                          double* delta_c);
// model cost change + candidate cost in one observation pass:
//  partial[grid][3] = { sum -(m.(r+m/2)), sum rc^2, nonfinite }
void launch_candidate(hipStream_t s, const DevView& v, const double* J, const double* r,
                      const double* delta_p, const double* delta_c, const double* points_c,
                      const double* camtab_c, double* partial, int grid);
// gradient norms over points: partial[grid][3] = {max |x-(x-g)|, sum (x-(x-g))^2, sum x^2}
void launch_grad_points(hipStream_t s, int NP, const double* x, const double* g /*[3][NP]*/,
                        double* partial, int grid);

// ---- dense Cholesky (dab_chol.hip) -------------------------------------------------------
// Factor the (n+1)x(n+1) augmented lower matrix [S b; b^T *] in place (row-major, ld = lds):
// on success the first n rows hold L and row n holds z = L^-1 b. Then solve L^T y = z into y.
// Returns 0 / nonzero (not PD). `work` needs >= 64 ints.
struct CholCtx;
CholCtx* chol_create();
void chol_destroy(CholCtx*);
int chol_factor_solve(CholCtx* c, hipStream_t s, int n, double* A, int lda, double* y, int* d_flag);

int grid_for(int n, int block, int cap);

}  // namespace dab
