// dab_solver.hip — C ABI + device-resident trust-region LM driver.
//
// Replaces ceres::Solve(options{DENSE_SCHUR}, &problem, &summary) as called by
// solve() at src/sfm.cc:31-75. The minimizer mirrors Ceres' TrustRegionMinimizer +
// LevenbergMarquardtStrategy: Jacobi scaling computed at iteration 0,
// LM diagonal clamp [1e-6, 1e32] / radius, step quality = actual/model decrease,
// radius /= max(1/3, 1-(2q-1)^3) on accept, /= decrease_factor (doubling) on reject,
// parameter / function / gradient tolerance tests in Ceres' order, five consecutive
// invalid steps => FAILURE, final_cost = min over iteration costs. The step solves
// (Js^T Js + D^2) y = Js^T r exactly: points are eliminated per point (3x3 Cholesky)
// and the reduced camera system is factored densely (dab_chol.hip) — DENSE_SCHUR.
//
// Multi-GPU: one process per GPU, observations sharded by point; the camera-side
// normal-equation pieces (U, g_c, the reduced system S and its rhs) and the scalar
// reductions are all-reduced with RCCL over xGMI; every rank then factors the same S
// and back-substitutes its own points.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <iterator>
#include <array>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "dab_devmem.h"
#include "dab_internal.h"
#include "dab_kernels.h"
#include "dab_p2p.h"
#include "dab_setup.h"

using namespace dab;

#define HIP_OK(expr)                                                                           \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      return set_error(DAB_E_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_));      \
  } while (0)
#define NCCL_OK(expr)                                                                          \
  do {                                                                                         \
    ncclResult_t e_ = (expr);                                                                  \
    if (e_ != ncclSuccess)                                                                     \
      return set_error(DAB_E_COMM, std::string(#expr) + ": " + ncclGetErrorString(e_));       \
  } while (0)
#define CHECK_RC(expr)       \
  do {                       \
    int rc_ = (expr);        \
    if (rc_ != 0) return rc_; \
  } while (0)

namespace dab {
namespace {
std::mutex& cache_mu() {
  static std::mutex* m = new std::mutex();  // never destroyed: handles may outlive static teardown
  return *m;
}
std::map<int, std::vector<hipStream_t>>& stream_cache() {
  static auto* c = new std::map<int, std::vector<hipStream_t>>();
  return *c;
}
std::map<size_t, std::vector<void*>>& pinned_cache() {
  static auto* c = new std::map<size_t, std::vector<void*>>();
  return *c;
}
}  // namespace
hipStream_t stream_take(int device) {
  {
    std::lock_guard<std::mutex> lk(cache_mu());
    auto& v = stream_cache()[device];
    while (!v.empty()) {
      hipStream_t s = v.back();
      v.pop_back();
      const hipError_t q = hipStreamQuery(s);  // a stream left in an error state is not reused
      if (q == hipSuccess || q == hipErrorNotReady) return s;
      (void)hipGetLastError();
      (void)hipStreamDestroy(s);
    }
  }
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  return s;
}
void stream_give(int device, hipStream_t s) {
  if (!s) return;
  if (hipStreamSynchronize(s) != hipSuccess) {  // a stream in an error state is not reused
    (void)hipStreamDestroy(s);
    return;
  }
  std::lock_guard<std::mutex> lk(cache_mu());
  stream_cache()[device].push_back(s);
}
void* pinned_take(size_t bytes) {
  {
    std::lock_guard<std::mutex> lk(cache_mu());
    auto& v = pinned_cache()[bytes];
    if (!v.empty()) {
      void* p = v.back();
      v.pop_back();
      return p;
    }
  }
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes) != hipSuccess) return nullptr;
  return p;
}
void pinned_give(void* p, size_t bytes) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(cache_mu());
  pinned_cache()[bytes].push_back(p);
}
}  // namespace dab

extern "C" int dab_release_caches(void) {
  std::lock_guard<std::mutex> lk(dab::cache_mu());
  // only idle cached objects live here (a handle takes its streams out of the cache and
  // gives them back on destroy), so live handles are unaffected; each device's streams are
  // destroyed with that device current
  int cur = 0;
  const bool have_cur = hipGetDevice(&cur) == hipSuccess;
  for (auto& kv : dab::stream_cache()) {
    if (kv.second.empty()) continue;
    (void)hipSetDevice(kv.first);
    for (hipStream_t s : kv.second) (void)hipStreamDestroy(s);
  }
  if (have_cur) (void)hipSetDevice(cur);
  dab::stream_cache().clear();
  for (auto& kv : dab::pinned_cache())
    for (void* p : kv.second) (void)hipHostFree(p);
  dab::pinned_cache().clear();
  return 0;
}

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Host set-up runs again after every filterPoint3d round (sfm.cc:118-127), so its
// O(observations) passes are spread over host threads. Every pass below gives the same
// result as its sequential form (each thread owns a contiguous index range; the counting
// sorts are stable: per-thread bucket counts are offset in (bucket, thread) order).
int setup_threads() {
  static const int t = [] {
    int n = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(n, 16));
  }();
  return t;
}
template <class F>
void par_for(long long n, F f, long long grain = 65536) {  // f(begin, end, thread), contiguous ranges
  const int T = (int)std::min<long long>(setup_threads(), std::max(1LL, n / grain));
  if (T <= 1) {
    f(0LL, n, 0);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) th.emplace_back([&, t] { f(n * t / T, n * (t + 1) / T, t); });
  for (auto& x : th) x.join();
}
// vectors whose elements are default-initialised (no zero fill): the large set-up arrays
// are first touched by the parallel passes that fill them, not by one thread
template <class T>
struct NoInit : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = NoInit<U>;
  };
  NoInit() = default;
  template <class U>
  NoInit(const NoInit<U>&) {}
  template <class U, class... Args>
  void construct(U* p, Args&&... args) {
    ::new ((void*)p) U(std::forward<Args>(args)...);
  }
  template <class U>
  void construct(U* p) {
    ::new ((void*)p) U;
  }
};
template <class T>
using big_vec = std::vector<T, NoInit<T>>;

// Pair-major chunks: a pair of n records is cut into ceil(n / most) equal pieces (the last
// one shorter by less than one per piece), not into full chunks and a ragged remainder:
// every chunk's work-group then runs about the same number of iterations per lane
static size_t pair_piece(size_t n, int most) {
  const size_t m = (size_t)std::max(1, most), parts = std::max<size_t>(1, (n + m - 1) / m);
  return std::max<size_t>(1, (n + parts - 1) / parts);
}

// stable counting sort of [0, n) by key(i) in [0, nb): out[pos] = i; start[nb + 1] = bucket
// offsets. key(i) < 0 drops i.
template <class K, class V>
void bucket_sort(long long n, int nb, K key, V& out, std::vector<long long>& start) {
  const int T = (int)std::min<long long>(setup_threads(), std::max(1LL, n / 65536));
  std::vector<std::vector<int>> cnt(T, std::vector<int>((size_t)nb, 0));
  std::vector<std::thread> th;
  auto range = [&](int t) { return std::make_pair(n * t / T, n * (t + 1) / T); };
  auto count = [&](int t) {
    auto r = range(t);
    for (long long i = r.first; i < r.second; ++i) {
      const int k = key(i);
      if (k >= 0) cnt[t][k]++;
    }
  };
  if (T > 1) {
    for (int t = 0; t < T; ++t) th.emplace_back(count, t);
    for (auto& x : th) x.join();
    th.clear();
  } else {
    count(0);
  }
  start.assign((size_t)nb + 1, 0);
  long long acc = 0;
  for (int b = 0; b < nb; ++b) {
    start[b] = acc;
    for (int t = 0; t < T; ++t) {
      const int c = cnt[t][b];
      cnt[t][b] = (int)acc;  // thread t's first position in bucket b
      acc += c;
    }
  }
  start[nb] = acc;
  out.resize((size_t)acc);
  auto place = [&](int t) {
    auto r = range(t);
    std::vector<int>& pos = cnt[t];
    for (long long i = r.first; i < r.second; ++i) {
      const int k = key(i);
      if (k >= 0) out[pos[k]++] = (int)i;
    }
  };
  if (T > 1) {
    for (int t = 0; t < T; ++t) th.emplace_back(place, t);
    for (auto& x : th) x.join();
  } else {
    place(0);
  }
}

// scalar slots of the per-handle scalar buffer
enum Slot {
  S_COST = 0,      // sum r^2 at x
  S_COST_BAD,      // non-finite residuals at x
  S_GMAX_P,        // max |x-(x-g)| over points
  S_GNORM_P,       // sum (x-(x-g))^2 over points
  S_XNORM_P,       // sum x^2 over points
  S_MODEL,         // model cost change
  S_CAND,          // sum r^2 at candidate
  S_CAND_BAD,      // non-finite residuals at candidate
  S_STEP_P,        // sum (x - xc)^2 over points
  S_XCNORM_P,      // sum xc^2 over points
  S_CAM0,          // 5 camera slots (launch_cam_norms)
  S_TIME = S_CAM0 + 5,  // solver wall-clock (max over ranks)
  S_END,
  // fixed-point cost shards of the prefetch point kernel (uint64 bit patterns: sum r^2
  // integer part, fraction * 2^52, non-finite count per shard; cost_fx_add)
  S_CFX = 16,  // two sets of kFxWords, alternating between passes
  S_XERR = S_CFX + 2 * kFxWords,  // k_eval_bal's error word (uint32 bits; 0 = ok)
  S_NSLOTS
};

// Device buffers of one problem come from a Dev (dab_devmem.h): dab_set_problem releases
// them all into a pool instead of freeing them, and an allocation takes the smallest pooled
// block that holds it without wasting more than half (or 1 MiB), so the sfm.cc loop's
// re-set-up after every filter round (the same problem, a little smaller) finds its ~50
// buffers there instead of paying a hipMalloc / hipFree pair each. A pooled block unused
// through one whole set-up and solve cycle is freed at the next release. The stream is
// synchronised before a release (dab_set_problem), so no queued kernel still reads a block
// that gets reused.

template <class T, class A>
int upload(T** dptr, Dev& dev, const std::vector<T, A>& h, hipStream_t s) {
  CHECK_RC(dev.alloc(dptr, h.size()));
  if (!h.empty()) HIP_OK(hipMemcpyAsync(*dptr, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, s));
  return 0;
}

// Tuning / test knobs from the environment, read once when the handle is created (never
// on a launch path). Unset = the production default.
struct Knobs {
  int chunk = 0;            // DAB_CHUNK: entries per camera-side reduction chunk (0: kChunk)
  int xchunk = 0;           // DAB_XCHUNK: most entries per pair-major chunk (0: kPairChunk)
  int pair_eval = -1;       // DAB_PAIR_EVAL=0: rig camera side camera-major + cross passes
  int eval_wps = INT_MIN;   // DAB_EVAL_WPS: point-kernel variant of the two-kernel pass
  int eval_fused = 1;       // DAB_EVAL_FUSED=0: two-kernel pass even where the fused one fits
  int eval_split = 0;       // DAB_EVAL_SPLIT=1: the multi-rank split schedule on one rank
  int pcg_fused = 1;        // DAB_PCG_FUSED=0
  int pcg_mf = 1;           // DAB_PCG_MF=0: stored-Y PCG even for small camera sets
  int cg_onewg = 0;         // DAB_CG_ONEWG=1: single-work-group CG update
  int bench_sample = 8;     // DAB_BENCH_SAMPLE: timing-event stride of dab_bench_eval_pass
  int schur_tiles = 1;      // DAB_SCHUR_TILES=0: explicit S from the pair tables even for small NC
  int tile_balance = 1;     // DAB_TILE_BALANCE=0: one work-group per tile and group of batches
  int tile_single = 1;      // DAB_TILE_SINGLE=0: k_schur_tiles with two LDS buffers (batches half as
                            // large, the next one in flight; round 6: one buffer, C5 EXACT 5.5 -> 5.2 ms)
  int tile_minb = 2;        // DAB_TILE_MINB: fewest batches per k_schur_tiles work-group (8 until round 6)
  int p2p = -1;             // DAB_P2P: one-shot xGMI all-reduce of small sums (-1 auto: RCCL handles
                            // only; 1 also on host-staged handles, the one-GPU rehearsal; 0 off)
  int setup_host = 0;       // DAB_SETUP_HOST=1: dab_set_problem's host passes instead of the device ones
  int eval_side = 0;        // DAB_EVAL_SIDE: 7 (test) a k_eval_bal frame wait that times out (the pass
                            // must fail with DAB_E_DEVICE on every rank). Builds with -DDAB_ABLATIONS
                            // also take the timing ablations (wrong results) 1 the point side only, 2
                            // the camera side only, 3 the tables only, 4 no tables or frames, 5 no
                            // point tables, 6 no camera frames; a release build refuses them
                            // (eval_side_ok: DAB_E_INVALID) instead of returning wrong sums
  int fused_tab = -1;       // DAB_FUSED_TAB: the fused pass reads the camera tables of the current x
                            // instead of building them in every work-group — -1 (default) when they
                            // exist already (the LM loop: the accepted candidate's tables), 1 always
                            // (building them first where they do not), 0 never
  void read() {
    auto get = [](const char* name, int& out) {
      if (const char* e = getenv(name)) out = atoi(e);
    };
    get("DAB_CHUNK", chunk);
    get("DAB_XCHUNK", xchunk);
    get("DAB_PAIR_EVAL", pair_eval);
    get("DAB_EVAL_WPS", eval_wps);
    get("DAB_EVAL_FUSED", eval_fused);
    get("DAB_EVAL_SPLIT", eval_split);
    get("DAB_PCG_FUSED", pcg_fused);
    get("DAB_PCG_MF", pcg_mf);
    get("DAB_CG_ONEWG", cg_onewg);
    get("DAB_BENCH_SAMPLE", bench_sample);
    get("DAB_SCHUR_TILES", schur_tiles);
    get("DAB_TILE_BALANCE", tile_balance);
    get("DAB_TILE_MINB", tile_minb);
    get("DAB_TILE_SINGLE", tile_single);
    get("DAB_P2P", p2p);
    get("DAB_FUSED_TAB", fused_tab);
    get("DAB_SETUP_HOST", setup_host);
    get("DAB_EVAL_SIDE", eval_side);
  }
  // the evaluation side this build accepts from DAB_EVAL_SIDE
  bool eval_side_ok() const {
#ifdef DAB_ABLATIONS
    return eval_side >= 0 && eval_side <= 7;
#else
    return eval_side == 0 || eval_side == 7;
#endif
  }
};

}  // namespace

struct dab_handle {
  Knobs knobs;
  int device = 0;
  int rank = 0, world = 1;
  hipStream_t stream = nullptr;
  ncclComm_t comm = nullptr;
  CholCtx* chol = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr;
  // multi-GPU: the camera-block all-reduce runs on its own stream, overlapping the
  // point-side kernel (ev_cam: camera blocks ready; ev_comm: all-reduce done)
  hipStream_t comm_stream = nullptr;
  hipEvent_t ev_cam = nullptr, ev_comm = nullptr;
  // bench bookkeeping
  double bench_jac_ms = 0, bench_asm_ms = 0, bench_pair_ms = 0;
  int bench_count = 0, bench_pending = 0, bench_pair_count = 0;
  // per-step events (dab_bench_eval_pass): start, point kernel start / end, end, and the
  // rig's pair-major camera kernel (k_eval_pair) start / end
  std::vector<std::array<hipEvent_t, 6>> bench_ev;
  std::vector<char> bench_pair_rec;  // per pending step: the pair events were recorded

  // ---- host-side problem structure ----
  bool have_problem = false;
  bool local_compose = false;       // some observation of this rank is composed (arc∘ring)
  bool host_entries = false;        // h_pt_ent_ptr / h_ent_* hold the entry lists (host set-up path)
  dab_problem prob{};               // caller's arrays (pointers valid until next set_problem)
  int N = 0, NP = 0, E = 0, NI = 0, NC = 0, NE = 0, nplanes = 18;
  bool any_compose = false;
  std::vector<int> perm;            // sorted obs -> caller's obs index
  std::vector<int> pt_of;           // local point -> caller's point id
  std::vector<int> ext_col;         // ext -> free camera column
  int nchunk = 0, nxchunk = 0, ncross = 0, nblk = 0, nslice = 0;
  int max_seg_chunks = 1, max_xseg_chunks = 1;  // largest chunk count of one camera / cross pair
  int NS = 0;  // observation slots (SELL-64, incl. padding)
  long long npairs = 0;
  int lds = 0;                      // leading dim of dense S
  bool schur_built = false;
  bool pcg_built = false;
  int nxlist = 0;
  std::vector<int> h_pt_ent_ptr;  // kept for build_schur_tables
  big_vec<int> h_ent_cam, h_ent_pos, h_ent_os;

  // ---- device buffers ----
  Dev dev{"problem buffers"};
  Dev setup_tmp{"set-up scratch"};  // the device set-up's scratch (released by the next set-up)
  Dev keep_dev{"kept buffers"};     // the Sticky buffers below (never released, re-sized by drop + alloc)
  DevView view{};
  int4* d_obs_idx = nullptr;
  double2* d_obs_xy = nullptr;
  // fused pass: packed 4-B slot records of the point waves (DevView::obs_e)
  int* d_obs_e = nullptr;
  int4* d_cm_idx = nullptr;
  double2* d_cm_xy = nullptr;
  int4* d_x_idx = nullptr;
  double2* d_x_xy = nullptr;
  int *d_slice_off = nullptr, *d_pt_ent_ptr = nullptr, *d_ent_os = nullptr, *d_ent_cam = nullptr,
      *d_ent_pt = nullptr, *d_ent_pos = nullptr, *d_cm_pt = nullptr, *d_ext_col = nullptr;
  int *d_chunk_beg = nullptr, *d_seg_chunk = nullptr;
  int2* d_chunk_uni = nullptr;
  int uni_affine = 0, uni_ox = 0, uni_oi = 0;  // chunk_uni[c] = (c + ox, c + oi) for every chunk
  unsigned* d_arrivals = nullptr;  // last-arriver counter of the point kernel (kept zeroed)
  int* d_chunk_lists = nullptr;  // uniform chunk ids, then the others
  ChunkLists chunks;
  int *d_xchunk_beg = nullptr, *d_xseg_chunk = nullptr;
  int2* d_cross_cam = nullptr;
  int2 *d_pairs = nullptr, *d_blk_cam = nullptr;
  int2* d_blk_zero = nullptr;  // lower blocks of S without pairs (one rank: zeroed directly)
  int nzero = 0;
  int* d_blk_pair_beg = nullptr;
  double* d_intr = nullptr;
  double *d_points = nullptr, *d_points_c = nullptr, *d_ext = nullptr, *d_ext_c = nullptr;
  double *d_camtab = nullptr, *d_camtab_c = nullptr;
  double* d_r = nullptr;
  double* d_Jfull = nullptr;  // parity API only (lazily allocated)
  double *d_V = nullptr, *d_g = nullptr, *d_scale_p = nullptr, *d_scale_c = nullptr;
  double *d_L = nullptr, *d_q = nullptr, *d_Y = nullptr, *d_Yp = nullptr;  // Y camera-/point-major
  double* d_Yrec = nullptr;  // EXPLICIT: Y as [NE][18] records for k_s_blocks (lazy)
  float *d_Y32c = nullptr, *d_Y32p = nullptr;                                 // pcg_fp32 (lazy)
  double* d_camred = nullptr;  // [Ucc NC*21 | gc NC*6 | Ux ncross*36] (all-reduced)
  double* d_partial = nullptr; // chunk partials (max of chunk counts * 36)
  double* d_xpartial = nullptr; // cross-block chunk partials
  // pair-major evaluation of the composed observations (launch_eval_pair): the other
  // entries' camera-major copy and chunks, and per camera its pair-chunk halves
  bool pair_eval = false;
  bool pair_uni_intr = false;  // one intrinsic per (arc, ring) pair: k_eval_pair's uniform tables
  double pair_bytes = 0.0, last_pair_ms = 0.0;  // k_eval_pair: algorithmic bytes per launch, bench time
  int nchunk2 = 0;
  int4* d_cm2_idx = nullptr;
  double2* d_cm2_xy = nullptr;
  int *d_chunk2_beg = nullptr, *d_seg2_chunk = nullptr, *d_xcam_ptr = nullptr, *d_xcam_list = nullptr;
  double *d_partial2 = nullptr, *d_xcpart = nullptr;
  double* d_spack = nullptr;   // [packed nblk*36 | ybc NC*6] (all-reduced)
  double* d_S = nullptr;
  // explicit S by fixed-point tiles (small camera sets, k_schur_tiles)
  bool schur_tiles = false;
  SchurTiles tiles{};
  int* d_kx = nullptr;                  // [6 NC] rhs row exponents
  double* d_sblk = nullptr;             // [nelem] Schur part of S by block (group sums, all-reduced)
  unsigned long long* d_rfx = nullptr;  // [6 NC] fixed-point rhs part (all-reduced as integers)
  double* d_yrec = nullptr;             // [nrec][18] Y of every record (this LM step)
  // implicit-Schur PCG (lazily allocated)
  double *d_pcg_b = nullptr, *d_pcg_r = nullptr, *d_pcg_z = nullptr, *d_pcg_p = nullptr, *d_pcg_q = nullptr,
         *d_pcg_w = nullptr, *d_pcg_Ad = nullptr, *d_pcg_Minv = nullptr, *d_pcg_red = nullptr,
         *d_pcg_t = nullptr;
  PcgState* d_pcg_state = nullptr;
  PcgState* h_pcg_state = nullptr;  // pinned
  int *d_xptr = nullptr, *d_xlist = nullptr, *d_run = nullptr;
  int* d_run_beg = nullptr;  // per chunk: its runs in d_run_rec
  int4* d_run_rec = nullptr;
  double *d_yc = nullptr, *d_dp = nullptr, *d_dc = nullptr;
  double* d_gpart = nullptr;   // grid partials
  double* d_scal = nullptr;    // S_NSLOTS
  int* d_flags = nullptr;      // [0] point factor fail, [1] chol fail
  double* h_scal = nullptr;    // pinned
  bool cost_fx_pending = false;  // fixed-point set fx_last holds the last evaluation's cost (read_scalars converts)
  int fx_last = 1;               // set of the last fixed-point pass (both sets start zeroed)
  int* h_flags = nullptr;      // pinned
  int red_grid = 1;
  bool fused_split = false;  // fused kernel as camera-side then point-side launches (world > 1)
  int eval_grid = 1;  // k_eval_points blocks (one SELL slice per block)
  int ncu = 256;      // compute units of the device
  int fused_grid = 0;  // > 0: single-pass PCG matvec (small camera systems)
  bool mf = false;     // matrix-free implicit Schur (no Y records; DAB_PCG_MF=0 disables)
  bool mf32 = false;   // this solve's matrix-free products in fp32 arithmetic (pcg_fp32)
  int mf_grid_n = 0;
  double* d_mf_partial = nullptr;
  const double* cg_wpart = nullptr;  // set by pcg_matvec: the partials the next CG update sums
  int pcg_hint = 2;    // CG iterations of the previous solve (first batch size)
  double* d_cg_partial = nullptr;  // multi-work-group CG update: grid partials + counter
  unsigned* d_cg_cnt = nullptr;
  double* d_fused_partial = nullptr;
  int eval_wps = 0;   // 0: LDS tables; else waves per slice (DAB_EVAL_WPS tuning knob)
  bool fused = false;  // evaluation pass as one launch (k_eval_bal; DAB_EVAL_FUSED=0 disables)

  // Buffers kept across dab_set_problem while the new problem's size fits: the dense S, the
  // camera step and the flags. The Cholesky's captured graph is keyed on their addresses, so
  // a problem re-set with the same camera count (the sfm.cc loop after every filter round)
  // replays the graph instead of capturing a new one.
  struct Sticky {
    void* p = nullptr;
    size_t cap = 0;
  };
  Sticky st_S, st_yc, st_flags;
  template <class T>
  int sticky(Sticky& st, T** out, size_t n) {
    const size_t bytes = std::max<size_t>(1, n) * sizeof(T);
    if (bytes > st.cap) {
      keep_dev.drop(st.p);
      st.p = nullptr;
      st.cap = 0;
      char* q = nullptr;
      CHECK_RC(keep_dev.alloc(&q, bytes));
      st.p = q;
      st.cap = bytes;
    }
    *out = static_cast<T*>(st.p);
    return 0;
  }

  ~dab_handle() {
    static const bool timing = getenv("DAB_SETUP_TIMING") != nullptr;
    double td = now_s();
    auto phase = [&](const char* what) {
      if (!timing) return;
      const double t = now_s();
      std::fprintf(stderr, "destroy %-22s %.2f ms (%zu live, %zu pooled blocks)\n", what, 1e3 * (t - td), dev.live.size(),
                   dev.pool.size());
      td = t;
    };
    phase("start");
    dev.clear();
    phase("device buffers");
    keep_dev.clear();
    pinned_give(h_scal, sizeof(double) * S_NSLOTS);
    pinned_give(h_flags, sizeof(int) * 4);
    pinned_give(h_pcg_state, sizeof(PcgState));
    if (h_stage) (void)hipHostFree(h_stage);
    phase("pinned");
    if (chol) chol_destroy(chol);
    phase("Cholesky context");
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (ev2) (void)hipEventDestroy(ev2);
    if (ev3) (void)hipEventDestroy(ev3);
    for (auto& e : bench_ev)
      for (hipEvent_t x : e) (void)hipEventDestroy(x);
    if (ev_cam) (void)hipEventDestroy(ev_cam);
    if (ev_comm) (void)hipEventDestroy(ev_comm);
    stream_give(device, comm_stream);
    p2p_destroy(p2p_main);
    p2p_destroy(p2p_comm);
    if (comm) ncclCommDestroy(comm);
    stream_give(device, stream);
  }

  unsigned* xerr() { return reinterpret_cast<unsigned*>(d_scal + S_XERR); }  // k_eval_bal's error word
  double* ug() { return d_camred; }  // [NC][27]: U upper-packed (21) | g_c (6)
  double* Ux() { return d_camred + (size_t)27 * NC; }
  size_t camred_count() const { return (size_t)27 * NC + (size_t)36 * ncross; }
  double* packed() { return d_spack; }
  double* ybc() { return d_spack + (size_t)36 * nblk; }
  size_t spack_count() const { return (size_t)36 * nblk + (size_t)6 * NC; }

  // one-shot xGMI all-reduce (dab_p2p.hip) of sums up to kP2pWords, one context per stream
  // (the main stream and the communication stream of the overlapped camera all-reduce)
  P2pComm* p2p_main = nullptr;
  P2pComm* p2p_comm = nullptr;
  static constexpr size_t kP2pWords = 65536;
  // an all-reduce on comm_stream can overlap the point-side kernel (RCCL or peer-to-peer)
  // rccl1: a one-rank handle on a real one-rank RCCL communicator (dab_create_dist with
  // world_size 1 and a unique id): every collective and the overlapped camera all-reduce run
  // through RCCL although they sum one rank, so the multi-GPU transport executes on one GPU
  bool rccl1 = false;
  bool coll() const { return world > 1 || rccl1; }
  bool can_overlap() const { return coll() && ((comm && !host_cb) || p2p_comm); }
  int allreduce_comm_stream(double* buf, size_t n) {
    if (p2p_comm && n <= kP2pWords) return p2p_allreduce_sum(p2p_comm, comm_stream, buf, n);
    if (!comm || host_cb) return set_error(DAB_E_STATE, "no collective for the communication stream");
    NCCL_OK(ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, comm, comm_stream));
    return 0;
  }

  // host-staged collective (dab_create_dist_host): rehearsal path, not the product path
  dab_host_allreduce_fn host_cb = nullptr;
  void* host_user = nullptr;
  double* h_stage = nullptr;  // pinned
  size_t stage_cap = 0;

  int stage(size_t n) {
    if (n <= stage_cap) return 0;
    if (h_stage) (void)hipHostFree(h_stage);
    h_stage = nullptr;
    stage_cap = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&h_stage), n * sizeof(double)) != hipSuccess)
      return set_error(DAB_E_NOMEM, "pinned staging allocation failed");
    stage_cap = n;
    return 0;
  }
  int host_allreduce(double* buf, size_t n, int op) {
    CHECK_RC(stage(n));
    HIP_OK(hipMemcpyAsync(h_stage, buf, n * sizeof(double), hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    if (host_cb(h_stage, (int64_t)n, op, host_user) != 0)
      return set_error(DAB_E_COMM, "host all-reduce callback failed");
    HIP_OK(hipMemcpyAsync(buf, h_stage, n * sizeof(double), hipMemcpyHostToDevice, stream));
    HIP_OK(hipStreamSynchronize(stream));
    return 0;
  }

  // exact integer sum over ranks of n uint64 words (the fixed-point cost); the host path
  // moves each word as three 22-bit pieces, which gloo's double sum adds exactly
  int allreduce_u64(uint64_t* buf, size_t n) {
    if (!coll() || n == 0) return 0;
    if (p2p_main && n <= kP2pWords)
      return p2p_allreduce_sum_u64(p2p_main, stream, reinterpret_cast<unsigned long long*>(buf), n);
    if (!host_cb) {
      NCCL_OK(ncclAllReduce(buf, buf, n, ncclUint64, ncclSum, comm, stream));
      return 0;
    }
    std::vector<uint64_t> tmp(n);
    CHECK_RC(stage(3 * n));
    HIP_OK(hipMemcpyAsync(tmp.data(), buf, n * sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    for (size_t i = 0; i < n; ++i)
      for (int k = 0; k < 3; ++k) h_stage[3 * i + k] = (double)((tmp[i] >> (22 * k)) & 0x3fffffull);
    if (host_cb(h_stage, (int64_t)(3 * n), 0, host_user) != 0)
      return set_error(DAB_E_COMM, "host all-reduce callback failed");
    for (size_t i = 0; i < n; ++i) {
      uint64_t v = 0;
      for (int k = 0; k < 3; ++k) v += (uint64_t)h_stage[3 * i + k] << (22 * k);
      tmp[i] = v;
    }
    HIP_OK(hipMemcpyAsync(buf, tmp.data(), n * sizeof(uint64_t), hipMemcpyHostToDevice, stream));
    HIP_OK(hipStreamSynchronize(stream));
    return 0;
  }
  unsigned long long* cost_fx(int set) const {
    return reinterpret_cast<unsigned long long*>(d_scal + S_CFX + (size_t)kFxWords * set);
  }
  // cost of the last evaluation pass summed over ranks (fixed point or double slots)
  int allreduce_cost() {
    if (cost_fx_pending) return allreduce_u64(reinterpret_cast<uint64_t*>(cost_fx(fx_last)), kFxWords);
    return allreduce(d_scal + S_COST, 2, ncclSum);
  }

  int allreduce(double* buf, size_t n, ncclRedOp_t op) {
    if (!coll() || n == 0) return 0;
    if (p2p_main && n <= kP2pWords && (op == ncclSum || op == ncclMax))
      return op == ncclSum ? p2p_allreduce_sum(p2p_main, stream, buf, n) : p2p_allreduce_max(p2p_main, stream, buf, n);
    if (host_cb) return host_allreduce(buf, n, op == ncclMax ? 1 : 0);
    NCCL_OK(ncclAllReduce(buf, buf, n, ncclDouble, op, comm, stream));
    return 0;
  }
  // max over ranks of small int flag arrays
  int allreduce_max_i32(int* buf, int n) {
    if (!coll() || n == 0) return 0;
    if (p2p_main) return p2p_allreduce_max_i32(p2p_main, stream, buf, (size_t)n);
    if (!host_cb) {
      NCCL_OK(ncclAllReduce(buf, buf, n, ncclInt32, ncclMax, comm, stream));
      return 0;
    }
    int tmp[16];
    if (n > 16) return set_error(DAB_E_INVALID, "flag all-reduce too large");
    CHECK_RC(stage(n));
    HIP_OK(hipMemcpyAsync(tmp, buf, n * sizeof(int), hipMemcpyDeviceToHost, stream));
    HIP_OK(hipStreamSynchronize(stream));
    for (int i = 0; i < n; ++i) h_stage[i] = tmp[i];
    if (host_cb(h_stage, n, 1, host_user) != 0) return set_error(DAB_E_COMM, "host all-reduce callback failed");
    for (int i = 0; i < n; ++i) tmp[i] = (int)h_stage[i];
    HIP_OK(hipMemcpyAsync(buf, tmp, n * sizeof(int), hipMemcpyHostToDevice, stream));
    HIP_OK(hipStreamSynchronize(stream));
    return 0;
  }
};

// ------------------------------------------------------------------------------------
// lifecycle
// ------------------------------------------------------------------------------------
__global__ void k_scale_points(int NP, const double* __restrict__ V, double* __restrict__ sp, int on);
static int create_common(int device, dab_handle** out) {
  if (!out) return set_error(DAB_E_INVALID, "null handle pointer");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return set_error(DAB_E_DEVICE, "no HIP device available");
  if (device < 0 || device >= ndev) return set_error(DAB_E_INVALID, "device ordinal out of range");
  HIP_OK(hipSetDevice(device));
  // Host waits spin (the solver's host round trips are latency-critical: read_scalars every
  // LM iteration). With the runtime's default the waits after a burst of short kernels
  // (the device set-up) fell back to blocking, and the first synchronisation of the
  // following solve took 10-25 ms for 10 us of device work. DAB_SCHEDULE_BLOCKING=1 keeps
  // the default.
  // The flag is process-wide (every host wait of the embedding process spins): dab.h says so.
  // A runtime that refuses it (flags fixed once the device's context exists) keeps its
  // default; that is reported once on stderr, not as an error.
  if (!getenv("DAB_SCHEDULE_BLOCKING")) {
    const hipError_t fe = hipSetDeviceFlags(hipDeviceScheduleSpin);
    static bool warned = false;
    if (fe != hipSuccess && !warned) {
      warned = true;
      fprintf(stderr, "dab: hipSetDeviceFlags(hipDeviceScheduleSpin) not applied (%s); host waits keep the "
                      "runtime's scheduling\n", hipGetErrorString(fe));
    }
  }
  static const bool timing = getenv("DAB_SETUP_TIMING") != nullptr;
  double tc = now_s();
  auto phase = [&](const char* what) {
    if (!timing) return;
    const double t = now_s();
    std::fprintf(stderr, "create %-24s %.2f ms\n", what, 1e3 * (t - tc));
    tc = t;
  };
  dab_handle* h = new dab_handle();
  h->device = device;
  h->knobs.read();
  if (!(h->stream = stream_take(device))) {
    delete h;
    return set_error(DAB_E_DEVICE, "hipStreamCreate failed");
  }
  phase("stream");
  h->chol = chol_create();
  phase("Cholesky context");
  if (!h->chol) {
    delete h;
    return set_error(DAB_E_DEVICE, "Cholesky context creation failed");
  }
  // an allocation that fails in one allocator first empties the others' idle pools
  h->keep_dev.donors = {&h->dev, &h->setup_tmp};
  chol_mem(h->chol)->donors = {&h->dev, &h->setup_tmp};
  h->dev.donors = {&h->setup_tmp};
  if (hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess ||
      hipEventCreate(&h->ev2) != hipSuccess || hipEventCreate(&h->ev3) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_cam, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_comm, hipEventDisableTiming) != hipSuccess ||
      !(h->comm_stream = stream_take(device))) {
    delete h;
    return set_error(DAB_E_DEVICE, "hipEventCreate failed");
  }
  if (!(h->h_scal = static_cast<double*>(pinned_take(sizeof(double) * S_NSLOTS))) ||
      !(h->h_flags = static_cast<int*>(pinned_take(sizeof(int) * 4)))) {
    delete h;
    return set_error(DAB_E_NOMEM, "hipHostMalloc failed");
  }
  phase("events, pinned");
  // every code object of the library loaded on this device now, once per process (the first
  // kernel launch of a translation unit would otherwise pay for it mid-solve)
  static bool warmed[64] = {};
  if (device < 64 && !warmed[device]) {
    warm_kernels();
    warm_chol();
    warm_pcg();
    warm_p2p();
    warm_setup();
    hipFuncAttributes a;
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(k_scale_points));
    warmed[device] = true;
    phase("code objects");
  }
  *out = h;
  return 0;
}

// DAB_DEV_GUARD=1: after an entry point's device work, every canary of the handle's
// allocators (problem buffers, set-up scratch, kept buffers, Cholesky scratch, and `extra`,
// an entry point's own temporaries) is read back; an overwritten one fails the call closed
// (DAB_E_DEVICE, the first block named in dab_last_error) instead of returning its result
static int guard_fail(dab_handle* h, const char* where, Dev* extra = nullptr) {
  if (!Dev::guard_on() || !h) return 0;
  (void)hipDeviceSynchronize();
  if (Dev::guard_mode() == 2 && std::strcmp(where, "dab_set_problem") == 0 && !h->dev.guards.empty()) {
    const unsigned char one = 1;  // the net's self-test: one byte past the first block
    (void)hipMemcpy(h->dev.guards.front().p, &one, 1, hipMemcpyHostToDevice);
  }
  std::string first;
  int bad = h->dev.guard_check(where, &first) + h->setup_tmp.guard_check(where, &first) +
            h->keep_dev.guard_check(where, &first) + chol_guard_check(h->chol, where, &first);
  if (extra) bad += extra->guard_check(where, &first);
  if (bad == 0) return 0;
  return set_error(DAB_E_DEVICE, "device guard: " + first +
                                     (bad > 1 ? " (and " + std::to_string(bad - 1) + " more)" : std::string()));
}

extern "C" int dab_create(int device, dab_handle** out) {
  clear_error();
  return create_common(device, out);
}

extern "C" int dab_comm_unique_id(uint8_t out_id[128]) {
  clear_error();
  if (!out_id) return set_error(DAB_E_INVALID, "null id buffer");
  ncclUniqueId id;
  NCCL_OK(ncclGetUniqueId(&id));
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  std::memcpy(out_id, &id, 128);
  return 0;
}

// The one-shot all-reduce contexts: every rank maps every peer's region (IPC handles
// gathered through the handle's own collective). Needs every pair of devices to be
// peer-accessible (one xGMI node); otherwise the sums stay on RCCL.
static int setup_p2p(dab_handle* h) {
  const bool want = h->knobs.p2p > 0 || (h->knobs.p2p < 0 && !h->host_cb);
  if (!want || h->world < 2 || h->world > kP2pMaxRanks) return 0;
  P2pAllgather gather;
  if (h->host_cb) {
    gather = [h](unsigned char* buf) -> int {
      const size_t n = (size_t)h->world * kP2pHandleBytes;
      if (h->stage(n) != 0) return -1;
      for (size_t i = 0; i < n; ++i) h->h_stage[i] = buf[i];
      if (h->host_cb(h->h_stage, (int64_t)n, 0, h->host_user) != 0) return -1;
      for (size_t i = 0; i < n; ++i) buf[i] = (unsigned char)h->h_stage[i];
      return 0;
    };
  } else {
    int ok = 1;  // peer access between this device and every other one of the node
    int ndev = 0;
    (void)hipGetDeviceCount(&ndev);
    for (int d = 0; d < ndev; ++d) {
      int a = 1;
      if (d != h->device && hipDeviceCanAccessPeer(&a, h->device, d) == hipSuccess && !a) ok = 0;
    }
    double f = ok ? 0.0 : 1.0;  // every rank must take the same branch
    double* d_f = nullptr;
    HIP_OK(hipMalloc(&d_f, sizeof(double)));
    HIP_OK(hipMemcpy(d_f, &f, sizeof(double), hipMemcpyHostToDevice));
    NCCL_OK(ncclAllReduce(d_f, d_f, 1, ncclDouble, ncclMax, h->comm, h->stream));
    HIP_OK(hipMemcpyAsync(&f, d_f, sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HIP_OK(hipStreamSynchronize(h->stream));
    (void)hipFree(d_f);
    if (f != 0.0) return 0;
    gather = [h](unsigned char* buf) -> int {
      const size_t n = (size_t)h->world * kP2pHandleBytes;
      unsigned char* d = nullptr;
      if (hipMalloc(&d, n) != hipSuccess) return -1;
      int rc = 0;
      if (hipMemcpy(d, buf, n, hipMemcpyHostToDevice) != hipSuccess ||
          ncclAllGather(d + (size_t)h->rank * kP2pHandleBytes, d, kP2pHandleBytes, ncclUint8, h->comm, h->stream) !=
              ncclSuccess ||
          hipMemcpyAsync(buf, d, n, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
          hipStreamSynchronize(h->stream) != hipSuccess)
        rc = -1;
      (void)hipFree(d);
      return rc;
    };
  }
  P2pComm* ctx[2] = {nullptr, nullptr};
  int rc = p2p_create_group(h->rank, h->world, dab_handle::kP2pWords, 2, gather, ctx);
  // a verified exchange on both contexts before the path is trusted (every rank runs it:
  // the calls are collective)
  for (int k = 0; k < 2 && rc == 0; ++k) rc = p2p_selftest(ctx[k], h->stream);
  // every rank must agree: if the contexts could not be set up or did not verify anywhere,
  // all ranks keep their sums on RCCL (or the host path) instead
  double bad = rc != 0 ? 1.0 : 0.0;
  if (h->host_cb) {
    CHECK_RC(h->stage(1));
    h->h_stage[0] = bad;
    if (h->host_cb(h->h_stage, 1, 1, h->host_user) != 0) return set_error(DAB_E_COMM, "host all-reduce failed");
    bad = h->h_stage[0];
  } else {
    double* d_f = nullptr;
    HIP_OK(hipMalloc(&d_f, sizeof(double)));
    HIP_OK(hipMemcpy(d_f, &bad, sizeof(double), hipMemcpyHostToDevice));
    NCCL_OK(ncclAllReduce(d_f, d_f, 1, ncclDouble, ncclMax, h->comm, h->stream));
    HIP_OK(hipMemcpyAsync(&bad, d_f, sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HIP_OK(hipStreamSynchronize(h->stream));
    (void)hipFree(d_f);
  }
  if (bad != 0.0) {
    // one line on stderr: a silent fallback would hide a platform whose peer mappings fail
    fprintf(stderr, "dab: rank %d: peer-to-peer all-reduce not verified (%s); sums stay on %s\n", h->rank,
            rc != 0 ? dab_last_error() : "a peer failed", h->host_cb ? "the host collective" : "RCCL");
    p2p_destroy(ctx[0]);
    p2p_destroy(ctx[1]);
    clear_error();
    return 0;
  }
  h->p2p_main = ctx[0];
  h->p2p_comm = ctx[1];
  return 0;
}

extern "C" int dab_create_dist(int device, int rank, int world_size, const uint8_t unique_id[128],
                               dab_handle** out) {
  clear_error();
  if (world_size < 1 || rank < 0 || rank >= world_size) return set_error(DAB_E_INVALID, "bad rank/world");
  if (world_size > 1 && !unique_id) return set_error(DAB_E_INVALID, "null unique id");
  CHECK_RC(create_common(device, out));
  dab_handle* h = *out;
  h->rank = rank;
  h->world = world_size;
  if (world_size == 1 && unique_id) {
    // one-rank RCCL communicator: the collectives execute (on one GPU) instead of returning
    ncclUniqueId id;
    std::memcpy(&id, unique_id, 128);
    ncclResult_t r = ncclCommInitRank(&h->comm, 1, id, 0);
    if (r != ncclSuccess) {
      std::string msg = std::string("ncclCommInitRank (one rank): ") + ncclGetErrorString(r);
      delete h;
      *out = nullptr;
      return set_error(DAB_E_COMM, msg);
    }
    h->rccl1 = true;
  }
  if (world_size > 1) {
    ncclUniqueId id;
    std::memcpy(&id, unique_id, 128);
    ncclResult_t r = ncclCommInitRank(&h->comm, world_size, id, rank);
    if (r != ncclSuccess) {
      std::string msg = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
      delete h;
      *out = nullptr;
      return set_error(DAB_E_COMM, msg);
    }
    if (setup_p2p(h) != 0) {
      delete h;
      *out = nullptr;
      return -1;
    }
  }
  return 0;
}

extern "C" int dab_create_dist_host(int device, int rank, int world_size, dab_host_allreduce_fn cb, void* user,
                                    dab_handle** out) {
  clear_error();
  if (world_size < 1 || rank < 0 || rank >= world_size) return set_error(DAB_E_INVALID, "bad rank/world");
  if (world_size > 1 && !cb) return set_error(DAB_E_INVALID, "null all-reduce callback");
  CHECK_RC(create_common(device, out));
  dab_handle* h = *out;
  h->rank = rank;
  h->world = world_size;
  h->host_cb = cb;
  h->host_user = user;
  if (world_size > 1 && setup_p2p(h) != 0) {
    delete h;
    *out = nullptr;
    return -1;
  }
  return 0;
}

extern "C" int dab_destroy(dab_handle* h) {
  clear_error();
  if (!h) return 0;
  (void)hipSetDevice(h->device);
  (void)hipStreamSynchronize(h->stream);
  static const bool timing = getenv("DAB_SETUP_TIMING") != nullptr;
  const double t0 = now_s();
  delete h;
  if (timing) std::fprintf(stderr, "destroy %.2f ms\n", 1e3 * (now_s() - t0));
  return 0;
}

// ------------------------------------------------------------------------------------
// problem setup: orderings and reduction tables (built once)
// ------------------------------------------------------------------------------------
static int validate(const dab_problem* p) {
  if (!p) return set_error(DAB_E_INVALID, "null problem");
  if (p->num_obs < 0 || p->num_points < 0 || p->num_ext < 0 || p->num_intr < 0)
    return set_error(DAB_E_INVALID, "negative size");
  if (p->num_obs > 0 && (!p->obs_xy || !p->obs_point || !p->obs_ext0 || !p->obs_ext1 || !p->obs_intr))
    return set_error(DAB_E_INVALID, "null observation array");
  if ((p->num_points > 0 && !p->points) || (p->num_ext > 0 && !p->ext) ||
      (p->num_intr > 0 && (!p->intr || !p->intr_nf || !p->intr_nk)))
    return set_error(DAB_E_INVALID, "null parameter array");
  for (int i = 0; i < p->num_intr; ++i) {
    if (p->intr_nf[i] < 1 || p->intr_nf[i] > 2) return set_error(DAB_E_INVALID, "intr_nf must be 1 or 2");
    if (p->intr_nk[i] < 0 || p->intr_nk[i] > 2) return set_error(DAB_E_INVALID, "intr_nk must be 0, 1 or 2");
  }
  return 0;
}
// per-observation index ranges (the host path; the device path checks them in su_count)
static int validate_obs(const dab_problem* p) {
  for (int o = 0; o < p->num_obs; ++o) {
    const int pt = p->obs_point[o], e0 = p->obs_ext0[o], e1 = p->obs_ext1[o], ii = p->obs_intr[o];
    if (pt < 0 || pt >= p->num_points || e0 < 0 || e0 >= p->num_ext || e1 < -1 || e1 >= p->num_ext ||
        ii < 0 || ii >= p->num_intr)
      return set_error(DAB_E_INVALID, "observation " + std::to_string(o) + " has an out-of-range index");
  }
  return 0;
}

// The host reference path of the set-up (DAB_SETUP_HOST=1; multi-rank problems and sizes
// setup_device_fits refuses): stable counting sorts and gathers on host threads, then the
// uploads. setup_device builds the same arrays on the GPU.
// whether the camera chunks' (ext, intr) pairs are an affine map of the chunk index (one
// chunk per free camera, both indices offset by a constant): the fused pass then computes them
static void set_uni_affine(dab_handle* h, const std::vector<int2>& cu) {
  h->uni_affine = 0;
  h->uni_ox = h->uni_oi = 0;
  if (cu.empty() || (int)cu.size() != h->NC) return;
  const int ox = cu[0].x, oi = cu[0].y;
  if (ox < 0 || oi < 0) return;
  for (size_t c = 0; c < cu.size(); ++c)
    if (cu[c].x != (int)c + ox || cu[c].y != (int)c + oi) return;
  h->uni_affine = 1;
  h->uni_ox = ox;
  h->uni_oi = oi;
}
static int setup_host(dab_handle* h, const dab_problem* p, const std::function<void(const char*)>& phase) {
  CHECK_RC(validate_obs(p));
  h->setup_tmp.clear();  // a previous device set-up's scratch (the host path needs none)
  const int N = p->num_obs;
  hipStream_t s = h->stream;
  // referenced points (local compact ids, in id order) and extrinsics
  std::vector<int> pt_local(p->num_points, -1);
  std::vector<char> pref(p->num_points, 0);
  std::vector<double> eref(std::max(1, p->num_ext), 0.0);
  h->any_compose = false;
  for (int o = 0; o < N; ++o) {
    pref[p->obs_point[o]] = 1;
    eref[p->obs_ext0[o]] = 1.0;
    if (p->obs_ext1[o] >= 0) {
      eref[p->obs_ext1[o]] = 1.0;
      h->any_compose = true;
    }
  }
  // device point order: referenced points by observation count, descending (stable by
  // id), so that the 64 points of one wave slice have similar track lengths (SELL-64)
  std::vector<int> pcount(p->num_points, 0);
  int maxcount = 0;
  for (int o = 0; o < N; ++o) maxcount = std::max(maxcount, ++pcount[p->obs_point[o]]);
  {  // counting sort by count, descending, stable by id (linear: set-up recurs per filter round)
    std::vector<int> start(maxcount + 2, 0);
    int npref = 0;
    for (int i = 0; i < p->num_points; ++i)
      if (pref[i]) {
        start[maxcount - pcount[i] + 1]++;
        ++npref;
      }
    for (int k = 0; k <= maxcount; ++k) start[k + 1] += start[k];
    h->pt_of.assign(npref, 0);
    for (int i = 0; i < p->num_points; ++i)
      if (pref[i]) h->pt_of[start[maxcount - pcount[i]]++] = i;
  }
  for (int l = 0; l < (int)h->pt_of.size(); ++l) pt_local[h->pt_of[l]] = l;
  h->NP = (int)h->pt_of.size();
  // the free camera set must agree on every rank
  if (h->world > 1) {
    double* d_tmp = nullptr;
    CHECK_RC(h->dev.alloc(&d_tmp, eref.size() + 1));
    eref.push_back(h->any_compose ? 1.0 : 0.0);
    HIP_OK(hipMemcpyAsync(d_tmp, eref.data(), eref.size() * sizeof(double), hipMemcpyHostToDevice, s));
    CHECK_RC(h->allreduce(d_tmp, eref.size(), ncclMax));
    HIP_OK(hipMemcpyAsync(eref.data(), d_tmp, eref.size() * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    h->any_compose = eref.back() != 0.0;
    eref.pop_back();
  }
  h->ext_col.assign(p->num_ext, -1);
  h->NC = 0;
  for (int e = 0; e < p->num_ext; ++e) {
    const bool is_const = p->freeze_camera || (p->ext_const && p->ext_const[e]);
    if (eref[e] != 0.0 && !is_const) h->ext_col[e] = h->NC++;
  }
  const int NP = h->NP, NC = h->NC;
  h->nplanes = h->any_compose ? 30 : 18;
  phase("points, cameras");

  // Observation slots, SELL-64: slice sl holds local points [64 sl, 64 sl + 64); the k-th
  // observation (caller order) of the slice's lane-l point sits at slice_off[sl] + 64 k + l,
  // slices padded to their longest track (padding slots: point -1). One wave walks a
  // slice with every load coalesced and reduces V, g per lane with no cross-lane work.
  std::vector<int> cnt(NP + 1, 0);
  big_vec<int> by_pt;
  {
    std::vector<long long> st;
    bucket_sort(N, NP, [&](long long o) { return pt_local[p->obs_point[o]]; }, by_pt, st);
    for (int i = 0; i <= NP; ++i) cnt[i] = (int)st[i];
  }
  h->nslice = (NP + 63) / 64;
  std::vector<int> slice_off(h->nslice + 1, 0);
  for (int sl = 0; sl < h->nslice; ++sl) {
    const int p0 = 64 * sl;
    const int len = cnt[p0 + 1] - cnt[p0];  // longest track of the slice (sorted)
    slice_off[sl + 1] = slice_off[sl] + 64 * len;
  }
  const int NS = slice_off[h->nslice];
  h->NS = NS;
  h->perm.resize(NS);
  big_vec<int4> obs_idx(NS);
  big_vec<double2> obs_xy(NS);
  // entries (observation slots on free cameras), point-major: counted per point first
  std::vector<int> pt_ent_ptr(NP + 1, 0);
  par_for(64LL * h->nslice, [&](long long b, long long e, int) {
    for (int pt = (int)b; pt < (int)e; ++pt) {
      const int sl = pt / 64, lane = pt % 64;
      const int len = pt < NP ? cnt[pt + 1] - cnt[pt] : 0;
      for (int k = len; k < (slice_off[sl + 1] - slice_off[sl]) / 64; ++k) {  // padding slots
        const int slot = slice_off[sl] + 64 * k + lane;
        h->perm[slot] = -1;
        obs_idx[slot] = make_int4(-1, 0, -1, 0);
        obs_xy[slot] = make_double2(0.0, 0.0);
      }
      if (pt >= NP) continue;
      int ne = 0;
      for (int k = 0; k < len; ++k) {
        const int slot = slice_off[sl] + 64 * k + lane;
        const int o = by_pt[cnt[pt] + k];
        h->perm[slot] = o;
        obs_idx[slot] = make_int4(pt, p->obs_ext0[o], p->obs_ext1[o], p->obs_intr[o]);
        obs_xy[slot] = make_double2(p->obs_xy[2 * (size_t)o], p->obs_xy[2 * (size_t)o + 1]);
        ne += p->obs_ext0[o] >= 0 && h->ext_col[p->obs_ext0[o]] >= 0;
        ne += p->obs_ext1[o] >= 0 && h->ext_col[p->obs_ext1[o]] >= 0;
      }
      pt_ent_ptr[pt + 1] = ne;
    }
  });
  for (int pt = 0; pt < NP; ++pt) pt_ent_ptr[pt + 1] += pt_ent_ptr[pt];
  h->NE = pt_ent_ptr[NP];
  big_vec<int> ent_os(h->NE), ent_cam(h->NE), ent_pt(h->NE);
  par_for(NP, [&](long long b, long long e, int) {
    for (int pt = (int)b; pt < (int)e; ++pt) {
      const int sl = pt / 64, lane = pt % 64;
      int q = pt_ent_ptr[pt];
      for (int k = 0; k < cnt[pt + 1] - cnt[pt]; ++k) {
        const int s2 = slice_off[sl] + 64 * k + lane;
        for (int slot = 0; slot < 2; ++slot) {
          const int ex = slot ? obs_idx[s2].z : obs_idx[s2].y;
          if (ex < 0 || h->ext_col[ex] < 0) continue;
          ent_os[q] = 2 * s2 + slot;
          ent_cam[q] = h->ext_col[ex];
          ent_pt[q] = pt;
          ++q;
        }
      }
    }
  });
  phase("slots, entries");
  const int NE = h->NE;

  // camera-major entry lists, chunked (deterministic two-level reductions)
  big_vec<int> cam_ent;
  std::vector<int> cam_cnt(NC + 1, 0);
  {
    std::vector<long long> st;
    bucket_sort(NE, NC, [&](long long e) { return ent_cam[e]; }, cam_ent, st);
    for (int c = 0; c <= NC; ++c) cam_cnt[c] = (int)st[c];
  }
  // entries per reduction chunk (one block each); DAB_CHUNK is a tuning knob
  const int chunk = std::max(64, h->knobs.chunk > 0 ? h->knobs.chunk : kChunk);
  std::vector<int> chunk_beg, seg_chunk(NC + 1, 0);
  for (int c = 0; c < NC; ++c) {
    seg_chunk[c] = (int)chunk_beg.size();
    for (int b = cam_cnt[c]; b < cam_cnt[c + 1]; b += chunk) chunk_beg.push_back(b);
  }
  seg_chunk[NC] = (int)chunk_beg.size();
  h->nchunk = (int)chunk_beg.size();
  h->max_seg_chunks = 1;
  for (int c = 0; c < NC; ++c) h->max_seg_chunks = std::max(h->max_seg_chunks, seg_chunk[c + 1] - seg_chunk[c]);
  chunk_beg.push_back(NE);
  // camera-major record positions of the entries, and per observation
  big_vec<int> ent_pos(NE), cm_pt(NE);
  par_for(NE, [&](long long b, long long e, int) {
    for (long long i = b; i < e; ++i) {
      ent_pos[cam_ent[i]] = (int)i;
      cm_pt[i] = ent_pt[cam_ent[i]];
    }
  });
  // runs of one point inside one camera's positions (rig: a point seen by one arc through
  // several rings has several entries of that camera); run[i] = run length at its first
  // position, 0 elsewhere. The diagonal S block needs (sum_run Y)(sum_run Y)^T.
  std::vector<int> run(NE, 0);
  par_for(NC, [&](long long b, long long e, int) {
    for (int c = (int)b; c < (int)e; ++c) {
      int i = cam_cnt[c];
      while (i < cam_cnt[c + 1]) {
        int j = i + 1;
        while (j < cam_cnt[c + 1] && cm_pt[j] == cm_pt[i]) ++j;
        run[i] = j - i;
        i = j;
      }
    }
  }, 1);
  // static camera-major copy of the entries' observation inputs (matrix-free camera passes)
  big_vec<int4> cm_idx(NE);
  // the runs of each chunk as records {first position, length, point, camera} in position
  // order (k_mf_diag_frame: its loads need no dependent index load; run_beg[nchunk + 1])
  std::vector<int> run_beg(h->nchunk + 1, 0);
  par_for(h->nchunk, [&](long long b, long long e, int) {
    for (int c = (int)b; c < (int)e; ++c) {
      int n = 0;
      for (int i = chunk_beg[c]; i < chunk_beg[c + 1]; ++i) n += run[i] > 0;
      run_beg[c + 1] = n;
    }
  }, 64);
  for (int c = 0; c < h->nchunk; ++c) run_beg[c + 1] += run_beg[c];
  big_vec<int4> run_rec(std::max(1, run_beg[h->nchunk]));
  big_vec<double2> cm_xy(NE);
  par_for(NE, [&](long long b, long long en, int) {
    for (long long i = b; i < en; ++i) {
      const int e = cam_ent[i], s2 = ent_os[e] >> 1;
      int4 id = obs_idx[s2];
      if (ent_os[e] & 1) id.w |= kSlotBit;
      cm_idx[i] = id;
      cm_xy[i] = obs_xy[s2];
    }
  });
  par_for(NC, [&](long long b, long long e, int) {
    for (int c = (int)b; c < (int)e; ++c)
      for (int q = seg_chunk[c]; q < seg_chunk[c + 1]; ++q) {
        int k = run_beg[q];
        for (int i = chunk_beg[q]; i < chunk_beg[q + 1]; ++i)
          if (run[i] > 0) run_rec[k++] = make_int4(i, run[i], cm_pt[i], c);
      }
  }, 1);
  // chunks whose entries all see one camera through one intrinsic (single-extrinsic
  // observations): the camera passes read that camera's tables once per block
  std::vector<int2> chunk_uni(h->nchunk, make_int2(-1, -1));
  par_for(h->nchunk, [&](long long b, long long e, int) {
    for (int q = (int)b; q < (int)e; ++q) {
      const int4 first = cm_idx[chunk_beg[q]];
      bool uni = first.z < 0 && !(first.w & kSlotBit);
      for (int i = chunk_beg[q]; uni && i < chunk_beg[q + 1]; ++i)
        uni = cm_idx[i].z < 0 && cm_idx[i].y == first.y && cm_idx[i].w == first.w;
      if (uni) chunk_uni[q] = make_int2(first.y, first.w);
    }
  }, 16);
  phase("camera-major");
  // arc∘ring cross blocks: composed observations whose two cameras are both free.
  // The pair table is the union over ranks so the all-reduced layout matches.
  // keys (c0 NC + c1) NS + s2 in increasing order: a counting sort by camera pair over the
  // slots in increasing order (linear; the comparison sort of 9M keys took ~1 s at C5)
  big_vec<long long> xkeys;
  if (h->any_compose && NC > 0) {
    // the two free cameras of a composed slot (-1: not a cross observation)
    auto cams_of = [&](long long s2) -> int2 {
      const int e1 = obs_idx[s2].z;
      if (e1 < 0 || obs_idx[s2].x < 0) return make_int2(-1, -1);
      const int c0 = h->ext_col[obs_idx[s2].y], c1 = h->ext_col[e1];
      if (c0 < 0 || c1 < 0) return make_int2(-1, -1);
      return make_int2(c0, c1);
    };
    // (c0, c1, slot) order by two stable NC-bucket passes (by c1, then by c0): counters of
    // NC per thread, not NC^2, and the 64-bit key below does not overflow
    big_vec<int> o1, o2;
    std::vector<long long> st1, st2;
    bucket_sort(NS, NC, [&](long long s2) { return cams_of(s2).y; }, o1, st1);
    bucket_sort((long long)o1.size(), NC, [&](long long j) { return cams_of(o1[j]).x; }, o2, st2);
    xkeys.resize(o2.size());
    par_for((long long)o2.size(), [&](long long b, long long e, int) {
      for (long long i = b; i < e; ++i) {
        const int s2 = o1[o2[i]];
        const int2 c = cams_of(s2);
        xkeys[i] = ((long long)c.x * NC + c.y) * (long long)NS + s2;
      }
    });
  }
  std::vector<long long> pairkeys;  // unique (c0*NC+c1)
  for (long long k : xkeys) {
    const long long pk = k / NS;
    if (pairkeys.empty() || pairkeys.back() != pk) pairkeys.push_back(pk);
  }
  if (h->world > 1 && h->any_compose && NC > 0) {
    // union of pair keys via an NC x NC bitmap all-reduce(max)
    std::vector<double> bm((size_t)NC * NC, 0.0);
    for (long long pk : pairkeys) bm[(size_t)pk] = 1.0;
    double* d_bm = nullptr;
    CHECK_RC(h->dev.alloc(&d_bm, bm.size()));
    HIP_OK(hipMemcpyAsync(d_bm, bm.data(), bm.size() * sizeof(double), hipMemcpyHostToDevice, s));
    CHECK_RC(h->allreduce(d_bm, bm.size(), ncclMax));
    HIP_OK(hipMemcpyAsync(bm.data(), d_bm, bm.size() * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    pairkeys.clear();
    for (size_t i = 0; i < bm.size(); ++i)
      if (bm[i] != 0.0) pairkeys.push_back((long long)i);
  }
  h->ncross = (int)pairkeys.size();
  std::vector<int2> cross_cam(h->ncross);
  for (int k = 0; k < h->ncross; ++k) cross_cam[k] = make_int2((int)(pairkeys[k] / NC), (int)(pairkeys[k] % NC));
  std::vector<int> xchunk_beg, xseg_chunk(h->ncross + 1, 0);
  big_vec<int4> x_idx(xkeys.size());
  big_vec<double2> x_xy(xkeys.size());
  {
    par_for((long long)xkeys.size(), [&](long long b, long long e, int) {
      for (long long i = b; i < e; ++i) {
        const int s2 = (int)(xkeys[i] % NS);
        x_idx[i] = obs_idx[s2];
        x_xy[i] = obs_xy[s2];
      }
    });
    std::vector<size_t> pbeg(h->ncross + 1, 0);
    std::vector<long long> pcnt(h->ncross, 0);
    size_t i = 0;
    for (int k = 0; k < h->ncross; ++k) {
      pbeg[k] = i;
      while (i < xkeys.size() && xkeys[i] / NS == pairkeys[k]) ++i;
      pcnt[k] = (long long)(i - pbeg[k]);
    }
    const int xchunk = std::max(64, h->knobs.xchunk > 0 ? h->knobs.xchunk : kPairChunk);
    for (int k = 0; k < h->ncross; ++k) {
      xseg_chunk[k] = (int)xchunk_beg.size();
      const size_t b = pbeg[k], piece = pair_piece((size_t)pcnt[k], xchunk);
      for (size_t q = b; q < b + (size_t)pcnt[k]; q += piece) xchunk_beg.push_back((int)q);
    }
    xseg_chunk[h->ncross] = (int)xchunk_beg.size();
    h->nxchunk = (int)xchunk_beg.size();
    h->max_xseg_chunks = 1;
    for (int k = 0; k < h->ncross; ++k)
      h->max_xseg_chunks = std::max(h->max_xseg_chunks, xseg_chunk[k + 1] - xseg_chunk[k]);
    xchunk_beg.push_back((int)xkeys.size());
  }

  // per-camera CSR of cross blocks for the implicit operator: code = 2 k + (camera is c1)
  std::vector<int> xptr(NC + 1, 0), xlist;
  {
    std::vector<std::vector<int>> per(NC);
    for (int k = 0; k < h->ncross; ++k) {
      per[cross_cam[k].x].push_back(2 * k);
      per[cross_cam[k].y].push_back(2 * k + 1);
    }
    for (int c = 0; c < NC; ++c) {
      xptr[c] = (int)xlist.size();
      xlist.insert(xlist.end(), per[c].begin(), per[c].end());
    }
    if (NC > 0) xptr[NC] = (int)xlist.size();
    h->nxlist = (int)xlist.size();
  }

  // pair-major evaluation (rig): the composed observations with both cameras free are
  // evaluated per (arc, ring) pair chunk; the remaining camera-major entries keep chunks
  // of their own, and every camera lists its halves of the pair chunks (increasing chunk)
  big_vec<int4> cm2_idx;
  big_vec<double2> cm2_xy;
  std::vector<int> chunk2_beg, seg2_chunk(NC + 1, 0), xcam_ptr(NC + 1, 0), xcam_list;
  h->pair_eval = h->nxchunk > 0 && pair_eval_fits(h->E, h->NI) && h->knobs.pair_eval != 0;
  if (h->pair_eval) {
    {  // algorithmic bytes of one k_eval_pair launch (dab_bench_pair_ms)
      std::vector<char> touched(NP, 0);
      long long npt = 0;
      for (long long k : xkeys) {
        const int p = obs_idx[(int)(k % NS)].x;
        if (p >= 0 && !touched[p]) {
          touched[p] = 1;
          ++npt;
        }
      }
      h->pair_bytes = (16.0 + 12.0) * (double)xkeys.size() + 24.0 * (double)npt + 90.0 * 8.0 * h->nxchunk;
      h->pair_uni_intr = true;
      for (size_t i = 1; i < x_idx.size() && h->pair_uni_intr; ++i)
        if (x_idx[i].y == x_idx[i - 1].y && x_idx[i].z == x_idx[i - 1].z && x_idx[i].w != x_idx[i - 1].w)
          h->pair_uni_intr = false;
    }
    // the entries that are not paired, per camera (counted, then filled in parallel)
    auto unpaired = [&](int i) {
      const int4 id = cm_idx[i];
      return !(id.z >= 0 && h->ext_col[id.y] >= 0 && h->ext_col[id.z] >= 0);
    };
    std::vector<int> c2cnt(NC + 1, 0);
    par_for(NC, [&](long long b, long long e, int) {
      for (int c = (int)b; c < (int)e; ++c) {
        int n2 = 0;
        for (int i = cam_cnt[c]; i < cam_cnt[c + 1]; ++i) n2 += unpaired(i);
        c2cnt[c + 1] = n2;
      }
    }, 1);
    for (int c = 0; c < NC; ++c) c2cnt[c + 1] += c2cnt[c];
    cm2_idx.resize(c2cnt[NC]);
    cm2_xy.resize(c2cnt[NC]);
    par_for(NC, [&](long long b, long long e, int) {
      for (int c = (int)b; c < (int)e; ++c) {
        int q = c2cnt[c];
        for (int i = cam_cnt[c]; i < cam_cnt[c + 1]; ++i)
          if (unpaired(i)) {
            cm2_idx[q] = cm_idx[i];
            cm2_xy[q] = cm_xy[i];
            ++q;
          }
      }
    }, 1);
    for (int c = 0; c < NC; ++c) {
      seg2_chunk[c] = (int)chunk2_beg.size();
      for (int q = c2cnt[c]; q < c2cnt[c + 1]; q += chunk) chunk2_beg.push_back(q);
    }
    seg2_chunk[NC] = (int)chunk2_beg.size();
    h->nchunk2 = (int)chunk2_beg.size();
    chunk2_beg.push_back((int)cm2_idx.size());
    std::vector<std::vector<int>> per(NC);
    for (int k = 0; k < h->ncross; ++k)
      for (int q = xseg_chunk[k]; q < xseg_chunk[k + 1]; ++q) {
        per[cross_cam[k].x].push_back(2 * q);
        per[cross_cam[k].y].push_back(2 * q + 1);
      }
    for (int c = 0; c < NC; ++c) {
      std::sort(per[c].begin(), per[c].end());
      xcam_ptr[c] = (int)xcam_list.size();
      xcam_list.insert(xcam_list.end(), per[c].begin(), per[c].end());
    }
    xcam_ptr[NC] = (int)xcam_list.size();
  }

  phase("pair-major");
  h->schur_built = false;
  h->schur_tiles = false;
  h->pcg_built = false;
  h->mf = h->mf32 = false;
  h->cg_wpart = nullptr;  // its buffer went with the previous problem's allocations
  h->fused_grid = 0;      // so did the single-pass product's partials
  h->mf_grid_n = 0;
  h->nblk = 0;
  h->nzero = 0;
  h->npairs = 0;

  // intrinsics: (cx, cy, fx, fy', k0, k1) with unused distortion terms zeroed
  std::vector<double> intr((size_t)kIntr * std::max(1, h->NI), 0.0);
  for (int i = 0; i < h->NI; ++i) {
    const double* K = p->intr + 6 * (size_t)i;
    double* o = &intr[(size_t)kIntr * i];
    o[0] = K[0];
    o[1] = K[1];
    o[2] = K[2];
    o[3] = p->intr_nf[i] == 2 ? K[3] : K[2];
    o[4] = p->intr_nk[i] >= 1 ? K[4] : 0.0;
    o[5] = p->intr_nk[i] >= 2 ? K[5] : 0.0;
  }
  std::vector<double> points((size_t)3 * NP);
  for (int i = 0; i < NP; ++i)
    for (int k = 0; k < 3; ++k) points[3 * (size_t)i + k] = p->points[3 * (size_t)h->pt_of[i] + k];
  std::vector<double> ext(p->ext, p->ext + 6 * (size_t)h->E);

  phase("host copies");
  // ---- upload ----
  Dev& d = h->dev;
  CHECK_RC(upload(&h->d_obs_idx, d, obs_idx, s));
  CHECK_RC(upload(&h->d_obs_xy, d, obs_xy, s));
  CHECK_RC(upload(&h->d_slice_off, d, slice_off, s));
  CHECK_RC(upload(&h->d_pt_ent_ptr, d, pt_ent_ptr, s));
  CHECK_RC(upload(&h->d_ent_os, d, ent_os, s));
  CHECK_RC(upload(&h->d_ent_cam, d, ent_cam, s));
  CHECK_RC(upload(&h->d_ent_pt, d, ent_pt, s));
  CHECK_RC(upload(&h->d_ext_col, d, h->ext_col, s));
  CHECK_RC(upload(&h->d_ent_pos, d, ent_pos, s));
  CHECK_RC(upload(&h->d_cm_pt, d, cm_pt, s));
  CHECK_RC(upload(&h->d_cm_idx, d, cm_idx, s));
  CHECK_RC(upload(&h->d_cm_xy, d, cm_xy, s));
  CHECK_RC(upload(&h->d_chunk_beg, d, chunk_beg, s));
  CHECK_RC(upload(&h->d_chunk_uni, d, chunk_uni, s));
  set_uni_affine(h, chunk_uni);
  CHECK_RC(d.alloc(&h->d_arrivals, 1));
  HIP_OK(hipMemsetAsync(h->d_arrivals, 0, sizeof(unsigned), s));
  {
    std::vector<int> lists;
    for (int q = 0; q < h->nchunk; ++q)
      if (chunk_uni[q].x >= 0) lists.push_back(q);
    const int nuni = (int)lists.size();
    for (int q = 0; q < h->nchunk; ++q)
      if (chunk_uni[q].x < 0) lists.push_back(q);
    CHECK_RC(upload(&h->d_chunk_lists, d, lists, s));
    h->chunks.nchunk = h->nchunk;
    h->chunks.nuni = nuni;
    h->chunks.ngen = h->nchunk - nuni;
    h->chunks.uni = h->d_chunk_lists;
    h->chunks.gen = h->d_chunk_lists + nuni;
  }
  CHECK_RC(upload(&h->d_seg_chunk, d, seg_chunk, s));
  CHECK_RC(upload(&h->d_x_idx, d, x_idx, s));
  CHECK_RC(upload(&h->d_x_xy, d, x_xy, s));
  CHECK_RC(upload(&h->d_xchunk_beg, d, xchunk_beg, s));
  CHECK_RC(upload(&h->d_xseg_chunk, d, xseg_chunk, s));
  CHECK_RC(upload(&h->d_cross_cam, d, cross_cam, s));
  CHECK_RC(upload(&h->d_xptr, d, xptr, s));
  CHECK_RC(upload(&h->d_run, d, run, s));
  CHECK_RC(upload(&h->d_run_beg, d, run_beg, s));
  CHECK_RC(upload(&h->d_run_rec, d, run_rec, s));
  CHECK_RC(upload(&h->d_xlist, d, xlist, s));
  if (h->pair_eval) {
    if (!cm2_idx.empty()) {
      CHECK_RC(upload(&h->d_cm2_idx, d, cm2_idx, s));
      CHECK_RC(upload(&h->d_cm2_xy, d, cm2_xy, s));
    }
    CHECK_RC(upload(&h->d_chunk2_beg, d, chunk2_beg, s));
    CHECK_RC(upload(&h->d_seg2_chunk, d, seg2_chunk, s));
    CHECK_RC(upload(&h->d_xcam_ptr, d, xcam_ptr, s));
    if (!xcam_list.empty()) CHECK_RC(upload(&h->d_xcam_list, d, xcam_list, s));
    CHECK_RC(d.alloc(&h->d_partial2, (size_t)std::max(1, h->nchunk2) * 27));
    CHECK_RC(d.alloc(&h->d_xcpart, (size_t)h->nxchunk * 54));
  }
  CHECK_RC(upload(&h->d_intr, d, intr, s));
  CHECK_RC(upload(&h->d_points, d, points, s));
  CHECK_RC(upload(&h->d_ext, d, ext, s));
  h->local_compose = false;
  for (int o = 0; o < N && !h->local_compose; ++o) h->local_compose = p->obs_ext1[o] >= 0;
  h->h_pt_ent_ptr = std::move(pt_ent_ptr);
  h->h_ent_cam = std::move(ent_cam);
  h->h_ent_pos = std::move(ent_pos);
  h->h_ent_os = std::move(ent_os);
  h->host_entries = true;
  return 0;
}

// Work buffers, launch geometry and the device view, common to both set-up paths.
static int setup_buffers(dab_handle* h, const std::function<void(const char*)>& phase) {
  hipStream_t s = h->stream;
  Dev& d = h->dev;
  const int NP = h->NP, NC = h->NC, NS = h->NS, NE = h->NE;
  CHECK_RC(d.alloc(&h->d_points_c, (size_t)3 * NP));
  CHECK_RC(d.alloc(&h->d_ext_c, (size_t)6 * h->E));
  CHECK_RC(d.alloc(&h->d_camtab, (size_t)kCamTab * h->E));
  CHECK_RC(d.alloc(&h->d_camtab_c, (size_t)kCamTab * h->E));
  CHECK_RC(d.alloc(&h->d_r, (size_t)2 * NS));
  h->d_Jfull = nullptr;
  CHECK_RC(d.alloc(&h->d_V, (size_t)6 * NP));
  CHECK_RC(d.alloc(&h->d_g, (size_t)3 * NP));
  CHECK_RC(d.alloc(&h->d_scale_p, (size_t)3 * NP));
  CHECK_RC(d.alloc(&h->d_scale_c, (size_t)6 * NC));
  CHECK_RC(d.alloc(&h->d_L, (size_t)6 * NP));
  CHECK_RC(d.alloc(&h->d_q, (size_t)4 * NP));
  CHECK_RC(d.alloc(&h->d_Y, (size_t)kYRec * NE));
  const size_t npm = (size_t)kYRec * std::max(1, h->NS) * (h->any_compose ? 2 : 1);
  CHECK_RC(d.alloc(&h->d_Yp, npm));
  h->d_Y32c = h->d_Y32p = nullptr;
  CHECK_RC(d.alloc(&h->d_camred, h->camred_count()));
  const size_t npart = std::max<size_t>({(size_t)h->nchunk * 27, (size_t)h->nxchunk * 36, (size_t)h->nchunk * 6, 16});
  CHECK_RC(d.alloc(&h->d_partial, npart));
  CHECK_RC(d.alloc(&h->d_xpartial, (size_t)std::max(1, h->nxchunk) * 36));
  CHECK_RC(h->sticky(h->st_yc, &h->d_yc, (size_t)6 * NC));
  CHECK_RC(d.alloc(&h->d_dp, (size_t)3 * NP));
  CHECK_RC(d.alloc(&h->d_dc, (size_t)6 * NC));
  h->red_grid = grid_for(std::max(h->NS, 3 * NP), 256, 1024);
  {
    // point-side kernel: LDS-staged camera tables when they fit (persistent grid, one
    // 1024-thread work-group per CU), else global tables (one block per slice).
    h->eval_wps = h->knobs.eval_wps != INT_MIN ? h->knobs.eval_wps : (eval_points_lds_fits(h->E) ? -2 : 4);
    int ncu = 256;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, h->device) == hipSuccess && prop.multiProcessorCount > 0)
      ncu = prop.multiProcessorCount;
    h->ncu = ncu;
    // LDS variants: one persistent work-group per CU (at most one per slice)
    // On several ranks the camera blocks' RCCL all-reduce runs during the point kernel. The
    // persistent point kernel (one 1024-thread, ~147-KB-LDS work-group per CU) would fill
    // every CU and hold the RCCL kernels off until it ends, so it leaves one CU per XCD
    // free for them (its slices are dealt round robin over whatever grid it gets).
    int pcus = ncu;
    // (a one-rank RCCL handle keeps the full grid: the same work-group partition, hence
    // bitwise the same sums, as dab_create)
    if (h->world > 1 && h->eval_wps <= 0) pcus = std::max(1, ncu - 8);
    h->eval_grid = h->eval_wps <= 0 ? std::max(1, std::min(pcus, h->nslice)) : std::max(1, h->nslice);
    h->fused = h->knobs.eval_fused != 0;
    h->fused_split = h->coll() || h->knobs.eval_split != 0;  // the split schedule on one rank too (tests)
  }
  CHECK_RC(d.alloc(&h->d_gpart, (size_t)std::max(h->red_grid, h->eval_grid) * 4));
  CHECK_RC(d.alloc(&h->d_scal, S_NSLOTS));
  CHECK_RC(h->sticky(h->st_flags, &h->d_flags, 4));
  HIP_OK(hipMemsetAsync(h->d_scal, 0, sizeof(double) * S_NSLOTS, s));  // both fixed-point cost sets start zeroed
  h->fx_last = 1;
  h->cost_fx_pending = false;
  HIP_OK(hipMemsetAsync(h->d_dc, 0, sizeof(double) * std::max(1, 6 * NC), s));
  HIP_OK(hipStreamSynchronize(s));

  DevView& v = h->view;
  v.N = h->NS;
  v.NP = NP;
  v.E = h->E;
  v.NC = NC;
  v.NI = h->NI;
  v.NE = NE;
  v.nslice = h->nslice;
  v.any_comp = h->local_compose ? 1 : 0;
  v.uni_affine = h->uni_affine;
  v.uni_ox = h->uni_ox;
  v.uni_oi = h->uni_oi;
  v.obs_idx = h->d_obs_idx;
  v.obs_xy = h->d_obs_xy;
  v.cm_idx = h->d_cm_idx;
  v.cm_xy = h->d_cm_xy;
  v.chunk_uni = h->d_chunk_uni;
  v.slice_off = h->d_slice_off;
  v.pt_ent_ptr = h->d_pt_ent_ptr;
  v.ent_os = h->d_ent_os;
  v.ent_cam = h->d_ent_cam;
  v.ent_pt = h->d_ent_pt;
  v.ent_pos = h->d_ent_pos;
  v.cm_pt = h->d_cm_pt;
  v.ext_col = h->d_ext_col;
  v.intr = h->d_intr;
  h->fused = h->fused && fused_eval_fits(v, h->nchunk, h->chunks.ngen, h->ncross, h->ncu);
  v.obs_e = nullptr;
  h->d_obs_e = nullptr;
  if (h->fused) {
    // packed 4-B slot records for the point waves (ext | intr << 16: fused_eval_fits keeps
    // E, NI <= kLdsCams)
    CHECK_RC(d.alloc(&h->d_obs_e, (size_t)std::max(1, NS)));
    su_obs_e(s, NS, h->d_obs_idx, h->d_obs_e);
    HIP_OK(hipStreamSynchronize(s));
    v.obs_e = h->d_obs_e;
  }
  HIP_OK(hipStreamSynchronize(s));
  phase("upload");
  h->have_problem = true;
  return 0;
}
// ---- set-up on the device (dab_setup.hip) ------------------------------------------------
// The same arrays as setup_host, built by rocPRIM radix sorts (stable: ties keep input
// order, exactly as the host's counting sorts) and gather / scatter kernels; only the
// camera-sized tables (chunks, cross pairs) are finished on the host. Multi-rank handles
// keep the host path: their free-camera and pair sets are unions over the ranks.
static int bits_for(long long maxval) {  // radix-sort end bit for keys in [0, maxval]
  int b = 1;
  while (b < 31 && (1LL << b) <= maxval) ++b;
  return b;
}
static bool setup_device_fits(dab_handle* h, const dab_problem* p) {
  if (h->world > 1) return false;
  const long long ncam = p->num_ext;  // NC <= num_ext; the pair key c0 NC + c1 must fit an int
  return ncam * ncam + 1 < (1LL << 30) && (long long)p->num_obs * 2 < (1LL << 30);
}
static int setup_device(dab_handle* h, const dab_problem* p, const std::function<void(const char*)>& phase) {
  hipStream_t s = h->stream;
  Dev& d = h->dev;
  // set-up scratch: kept until the next set-up (freeing it here stalled the solve's first
  // kernels by 10-25 ms)
  Dev& tmp = h->setup_tmp;
  tmp.release();
  const int N = p->num_obs, NPT = p->num_points, E = p->num_ext;
  // scratch for rocPRIM: sized by the largest query
  void* rtmp = nullptr;
  size_t rtmp_cap = 0;
  auto rp = [&](auto call) -> int {  // query the bytes, grow the scratch, run
    size_t bytes = 0;
    if (call(nullptr, &bytes) != 0) return set_error(DAB_E_DEVICE, "rocPRIM size query failed");
    if (bytes > rtmp_cap) {
      void* q = nullptr;
      CHECK_RC(tmp.alloc(reinterpret_cast<unsigned char**>(&q), bytes));
      rtmp = q;
      rtmp_cap = bytes;
    }
    if (call(rtmp, &bytes) != 0) return set_error(DAB_E_DEVICE, "rocPRIM pass failed");
    return 0;
  };
  auto d2h = [&](void* dst, const void* src, size_t bytes) -> int {
    if (bytes) HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
    return 0;
  };
  auto h2d = [&](void* dst, const void* src, size_t bytes) -> int {
    if (bytes) HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    return 0;
  };

  // ---- the caller's observation arrays ----
  int *r_pt = nullptr, *r_e0 = nullptr, *r_e1 = nullptr, *r_in = nullptr;
  double *r_xy = nullptr, *r_points = nullptr;
  CHECK_RC(tmp.alloc(&r_pt, N));
  CHECK_RC(tmp.alloc(&r_e0, N));
  CHECK_RC(tmp.alloc(&r_e1, N));
  CHECK_RC(tmp.alloc(&r_in, N));
  CHECK_RC(tmp.alloc(&r_xy, (size_t)2 * N));
  CHECK_RC(tmp.alloc(&r_points, (size_t)3 * std::max(1, NPT)));
  CHECK_RC(h2d(r_pt, p->obs_point, sizeof(int) * (size_t)N));
  CHECK_RC(h2d(r_e0, p->obs_ext0, sizeof(int) * (size_t)N));
  CHECK_RC(h2d(r_e1, p->obs_ext1, sizeof(int) * (size_t)N));
  CHECK_RC(h2d(r_in, p->obs_intr, sizeof(int) * (size_t)N));
  CHECK_RC(h2d(r_xy, p->obs_xy, sizeof(double) * 2 * (size_t)N));
  CHECK_RC(h2d(r_points, p->points, sizeof(double) * 3 * (size_t)NPT));
  phase("device: upload");

  // ---- counts, validation, referenced extrinsics ----
  int *pcount = nullptr, *eref_d = nullptr, *small = nullptr;  // small: [flags, maxcount, nref, nvalid, count, ...]
  CHECK_RC(tmp.alloc(&pcount, std::max(1, NPT)));
  CHECK_RC(tmp.alloc(&eref_d, std::max(1, E)));
  CHECK_RC(tmp.alloc(&small, 16));
  HIP_OK(hipMemsetAsync(pcount, 0, sizeof(int) * std::max(1, NPT), s));
  HIP_OK(hipMemsetAsync(eref_d, 0, sizeof(int) * std::max(1, E), s));
  HIP_OK(hipMemsetAsync(small, 0, sizeof(int) * 16, s));
  su_count(s, N, r_pt, r_e0, r_e1, r_in, NPT, E, p->num_intr, pcount, eref_d, small);
  if (NPT > 0)
    CHECK_RC(rp([&](void* t, size_t* b) { return su_max(t, b, pcount, small + 1, NPT, s); }));
  int hs[4] = {0, 0, 0, 0};
  std::vector<int> eref(std::max(1, E), 0);
  CHECK_RC(d2h(hs, small, sizeof(int) * 2));
  CHECK_RC(d2h(eref.data(), eref_d, sizeof(int) * (size_t)E));
  HIP_OK(hipStreamSynchronize(s));
  if (hs[0] & 1) {
    // the host check names the first offending observation
    CHECK_RC(validate_obs(p));
    return set_error(DAB_E_INVALID, "an observation has an out-of-range index");
  }
  h->local_compose = h->any_compose = (hs[0] & 2) != 0;
  const int maxcount = hs[1];

  // ---- device point order (count descending, stable by id) ----
  int *pk = nullptr, *pv = nullptr, *pk2 = nullptr, *pv2 = nullptr;
  CHECK_RC(tmp.alloc(&pk, std::max(1, NPT)));
  CHECK_RC(tmp.alloc(&pv, std::max(1, NPT)));
  CHECK_RC(tmp.alloc(&pk2, std::max(1, NPT)));
  CHECK_RC(tmp.alloc(&pv2, std::max(1, NPT)));
  su_point_keys(s, NPT, pcount, small + 1, pk, pv, small + 2);
  if (NPT > 0)
    CHECK_RC(rp([&](void* t, size_t* b) { return su_sort_pairs(t, b, pk, pk2, pv, pv2, NPT, bits_for(maxcount + 1), s); }));
  CHECK_RC(d2h(hs + 2, small + 2, sizeof(int)));
  HIP_OK(hipStreamSynchronize(s));
  const int NP = hs[2];
  h->NP = NP;
  h->pt_of.resize(NP);
  const int* pt_of_d = pv2;  // first NP sorted ids
  CHECK_RC(d2h(h->pt_of.data(), pt_of_d, sizeof(int) * (size_t)NP));
  int *pt_local = nullptr, *lcount = nullptr;
  CHECK_RC(tmp.alloc(&pt_local, std::max(1, NPT)));
  CHECK_RC(tmp.alloc(&lcount, NP + 1));
  su_point_local(s, NP, pt_of_d, pcount, pt_local, lcount);

  // ---- free cameras (host: E is small) ----
  h->ext_col.assign(E, -1);
  h->NC = 0;
  for (int e = 0; e < E; ++e) {
    const bool is_const = p->freeze_camera || (p->ext_const && p->ext_const[e]);
    if (eref[e] != 0 && !is_const) h->ext_col[e] = h->NC++;
  }
  const int NC = h->NC;
  h->nplanes = h->any_compose ? 30 : 18;
  CHECK_RC(upload(&h->d_ext_col, d, h->ext_col, s));
  phase("device: points, cameras");

  // ---- observations by point (stable), SELL-64 slots ----
  int *ok = nullptr, *ov = nullptr, *ok2 = nullptr, *by_pt = nullptr, *cnt = nullptr;
  CHECK_RC(tmp.alloc(&ok, std::max(1, N)));
  CHECK_RC(tmp.alloc(&ov, std::max(1, N)));
  CHECK_RC(tmp.alloc(&ok2, std::max(1, N)));
  CHECK_RC(tmp.alloc(&by_pt, std::max(1, N)));
  CHECK_RC(tmp.alloc(&cnt, NP + 1));
  su_obs_keys(s, N, r_pt, pt_local, ok, ov);
  if (N > 0)
    CHECK_RC(rp([&](void* t, size_t* b) { return su_sort_pairs(t, b, ok, ok2, ov, by_pt, N, bits_for(NP), s); }));
  CHECK_RC(rp([&](void* t, size_t* b) { return su_exclusive_scan(t, b, lcount, cnt, NP + 1, s); }));
  h->nslice = (NP + 63) / 64;
  const int nslice = h->nslice;
  int* slen = nullptr;
  CHECK_RC(tmp.alloc(&slen, nslice + 1));
  CHECK_RC(d.alloc(&h->d_slice_off, nslice + 1));
  su_slice_len(s, nslice, NP, lcount, slen);
  CHECK_RC(rp([&](void* t, size_t* b) { return su_exclusive_scan(t, b, slen, h->d_slice_off, nslice + 1, s); }));
  int NS = 0;
  CHECK_RC(d2h(&NS, h->d_slice_off + nslice, sizeof(int)));
  HIP_OK(hipStreamSynchronize(s));
  h->NS = NS;
  int *perm_d = nullptr, *ne = nullptr;
  CHECK_RC(d.alloc(&h->d_obs_idx, (size_t)std::max(1, NS)));
  CHECK_RC(d.alloc(&h->d_obs_xy, (size_t)std::max(1, NS)));
  CHECK_RC(tmp.alloc(&perm_d, std::max(1, NS)));
  CHECK_RC(tmp.alloc(&ne, NP + 1));
  su_slots(s, NP, nslice, h->d_slice_off, cnt, lcount, by_pt, r_e0, r_e1, r_in, r_xy, h->d_ext_col, h->d_obs_idx,
           h->d_obs_xy, perm_d, ne);
  h->perm.resize(NS);
  CHECK_RC(d2h(h->perm.data(), perm_d, sizeof(int) * (size_t)NS));
  // entries (free-camera slots), point-major
  CHECK_RC(d.alloc(&h->d_pt_ent_ptr, NP + 1));
  CHECK_RC(rp([&](void* t, size_t* b) { return su_exclusive_scan(t, b, ne, h->d_pt_ent_ptr, NP + 1, s); }));
  int NE = 0;
  CHECK_RC(d2h(&NE, h->d_pt_ent_ptr + NP, sizeof(int)));
  HIP_OK(hipStreamSynchronize(s));
  h->NE = NE;
  CHECK_RC(d.alloc(&h->d_ent_os, std::max(1, NE)));
  CHECK_RC(d.alloc(&h->d_ent_cam, std::max(1, NE)));
  CHECK_RC(d.alloc(&h->d_ent_pt, std::max(1, NE)));
  su_entries(s, NP, h->d_slice_off, lcount, h->d_obs_idx, h->d_ext_col, h->d_pt_ent_ptr, h->d_ent_os, h->d_ent_cam,
             h->d_ent_pt);
  phase("device: slots, entries");

  // ---- camera-major order (entries by camera, stable) ----
  int *ek = nullptr, *ev = nullptr, *pos_cam = nullptr, *cam_ent = nullptr, *cam_cnt_d = nullptr;
  CHECK_RC(tmp.alloc(&ev, std::max(1, NE)));
  CHECK_RC(tmp.alloc(&pos_cam, std::max(1, NE)));
  CHECK_RC(tmp.alloc(&cam_ent, std::max(1, NE)));
  CHECK_RC(tmp.alloc(&cam_cnt_d, NC + 1));
  ek = h->d_ent_cam;
  su_iota(s, NE, ev);
  if (NE > 0)
    CHECK_RC(rp([&](void* t, size_t* b) { return su_sort_pairs(t, b, ek, pos_cam, ev, cam_ent, NE, bits_for(NC), s); }));
  HIP_OK(hipMemsetAsync(cam_cnt_d, 0, sizeof(int) * (NC + 1), s));
  su_bounds(s, NE, pos_cam, NC, cam_cnt_d);
  std::vector<int> cam_cnt(NC + 1, 0);
  CHECK_RC(d2h(cam_cnt.data(), cam_cnt_d, sizeof(int) * (NC + 1)));
  HIP_OK(hipStreamSynchronize(s));
  // chunks (host: NC is small)
  const int chunk = std::max(64, h->knobs.chunk > 0 ? h->knobs.chunk : kChunk);
  std::vector<int> chunk_beg, seg_chunk(NC + 1, 0);
  for (int c = 0; c < NC; ++c) {
    seg_chunk[c] = (int)chunk_beg.size();
    for (int b = cam_cnt[c]; b < cam_cnt[c + 1]; b += chunk) chunk_beg.push_back(b);
  }
  seg_chunk[NC] = (int)chunk_beg.size();
  h->nchunk = (int)chunk_beg.size();
  h->max_seg_chunks = 1;
  for (int c = 0; c < NC; ++c) h->max_seg_chunks = std::max(h->max_seg_chunks, seg_chunk[c + 1] - seg_chunk[c]);
  chunk_beg.push_back(NE);
  const int nchunk = h->nchunk;
  CHECK_RC(upload(&h->d_chunk_beg, d, chunk_beg, s));
  CHECK_RC(upload(&h->d_seg_chunk, d, seg_chunk, s));
  CHECK_RC(d.alloc(&h->d_ent_pos, std::max(1, NE)));
  CHECK_RC(d.alloc(&h->d_cm_pt, std::max(1, NE)));
  CHECK_RC(d.alloc(&h->d_cm_idx, (size_t)std::max(1, NE)));
  CHECK_RC(d.alloc(&h->d_cm_xy, (size_t)std::max(1, NE)));
  su_camera_major(s, NE, cam_ent, h->d_ent_pt, h->d_ent_os, h->d_obs_idx, h->d_obs_xy, h->d_ent_pos, h->d_cm_pt,
                  h->d_cm_idx, h->d_cm_xy);
  CHECK_RC(d.alloc(&h->d_run, std::max(1, NE)));
  su_runs(s, NE, pos_cam, h->d_cm_pt, h->d_run);
  int* run_cnt = nullptr;
  CHECK_RC(tmp.alloc(&run_cnt, nchunk + 1));
  CHECK_RC(d.alloc(&h->d_run_beg, nchunk + 1));
  HIP_OK(hipMemsetAsync(run_cnt, 0, sizeof(int) * (nchunk + 1), s));
  su_chunk_runs(s, nchunk, h->d_chunk_beg, h->d_run, run_cnt);
  CHECK_RC(rp([&](void* t, size_t* b) { return su_exclusive_scan(t, b, run_cnt, h->d_run_beg, nchunk + 1, s); }));
  int nrun = 0;
  CHECK_RC(d2h(&nrun, h->d_run_beg + nchunk, sizeof(int)));
  HIP_OK(hipStreamSynchronize(s));
  CHECK_RC(d.alloc(&h->d_run_rec, (size_t)std::max(1, nrun)));
  su_chunk_run_rec(s, nchunk, h->d_chunk_beg, h->d_run, h->d_cm_pt, pos_cam, h->d_run_beg, h->d_run_rec);
  CHECK_RC(d.alloc(&h->d_chunk_uni, (size_t)std::max(1, nchunk)));
  su_chunk_uni(s, nchunk, h->d_chunk_beg, h->d_cm_idx, kSlotBit, h->d_chunk_uni);
  std::vector<int2> chunk_uni(nchunk);
  CHECK_RC(d2h(chunk_uni.data(), h->d_chunk_uni, sizeof(int2) * (size_t)nchunk));
  HIP_OK(hipStreamSynchronize(s));
  set_uni_affine(h, chunk_uni);
  phase("device: camera-major");

  // ---- pair-major copy of the composed observations (rig) ----
  std::vector<long long> pairkeys;
  std::vector<int> pair_cnt;
  int nx = 0;
  int* xslots = nullptr;
  if (h->any_compose && NC > 0) {
    // the (c0, c1) sort key c0 * NC + c1 (and its sentinel NC * NC) is a 32-bit int
    if ((long long)NC * NC > (long long)INT_MAX)
      return set_error(DAB_E_UNSUPPORTED, "composed observations with more than 46340 free cameras");
    int *xk = nullptr, *xv = nullptr, *xk2 = nullptr;
    CHECK_RC(tmp.alloc(&xk, std::max(1, NS)));
    CHECK_RC(tmp.alloc(&xv, std::max(1, NS)));
    CHECK_RC(tmp.alloc(&xk2, std::max(1, NS)));
    CHECK_RC(tmp.alloc(&xslots, std::max(1, NS)));
    su_cross_keys(s, NS, h->d_obs_idx, h->d_ext_col, NC, xk, xv, small + 3);
    CHECK_RC(rp([&](void* t, size_t* b) { return su_sort_pairs(t, b, xk, xk2, xv, xslots, NS, bits_for((long long)NC * NC), s); }));
    CHECK_RC(d2h(hs + 3, small + 3, sizeof(int)));
    HIP_OK(hipStreamSynchronize(s));
    nx = hs[3];
    if (nx > 0) {
      int *uk = nullptr, *uc = nullptr;
      CHECK_RC(tmp.alloc(&uk, nx));
      CHECK_RC(tmp.alloc(&uc, nx));
      CHECK_RC(rp([&](void* t, size_t* b) { return su_rle(t, b, xk2, uk, uc, small + 4, nx, s); }));
      int nr = 0;
      CHECK_RC(d2h(&nr, small + 4, sizeof(int)));
      HIP_OK(hipStreamSynchronize(s));
      std::vector<int> ukh(nr), uch(nr);
      CHECK_RC(d2h(ukh.data(), uk, sizeof(int) * (size_t)nr));
      CHECK_RC(d2h(uch.data(), uc, sizeof(int) * (size_t)nr));
      HIP_OK(hipStreamSynchronize(s));
      for (int k = 0; k < nr; ++k) {
        pairkeys.push_back(ukh[k]);
        pair_cnt.push_back(uch[k]);
      }
    }
  }
  h->ncross = (int)pairkeys.size();
  std::vector<int2> cross_cam(h->ncross);
  for (int k = 0; k < h->ncross; ++k) cross_cam[k] = make_int2((int)(pairkeys[k] / NC), (int)(pairkeys[k] % NC));
  std::vector<int> xchunk_beg, xseg_chunk(h->ncross + 1, 0);
  {
    int b = 0;
    const int xchunk = std::max(64, h->knobs.xchunk > 0 ? h->knobs.xchunk : kPairChunk);
    if (getenv("DAB_SETUP_TIMING")) {  // the pair sizes the chunk plan saw
      fprintf(stderr, "pair chunks: %d pairs, most %d records per chunk, counts", h->ncross, xchunk);
      for (int k = 0; k < h->ncross; ++k) fprintf(stderr, " %d", pair_cnt[k]);
      fprintf(stderr, "\n");
    }
    for (int k = 0; k < h->ncross; ++k) {
      xseg_chunk[k] = (int)xchunk_beg.size();
      const int piece = (int)pair_piece((size_t)pair_cnt[k], xchunk);
      for (int q = b; q < b + pair_cnt[k]; q += piece) xchunk_beg.push_back(q);
      b += pair_cnt[k];
    }
    xseg_chunk[h->ncross] = (int)xchunk_beg.size();
    h->nxchunk = (int)xchunk_beg.size();
    h->max_xseg_chunks = 1;
    for (int k = 0; k < h->ncross; ++k)
      h->max_xseg_chunks = std::max(h->max_xseg_chunks, xseg_chunk[k + 1] - xseg_chunk[k]);
    xchunk_beg.push_back(nx);
  }
  CHECK_RC(d.alloc(&h->d_x_idx, (size_t)std::max(1, nx)));
  CHECK_RC(d.alloc(&h->d_x_xy, (size_t)std::max(1, nx)));
  h->pair_eval = h->nxchunk > 0 && pair_eval_fits(h->E, h->NI) && h->knobs.pair_eval != 0;
  unsigned char* touched = nullptr;
  if (h->pair_eval) {
    CHECK_RC(tmp.alloc(&touched, std::max(1, NP)));
    HIP_OK(hipMemsetAsync(touched, 0, (size_t)std::max(1, NP), s));
  }
  su_cross_copy(s, nx, xslots, h->d_obs_idx, h->d_obs_xy, h->d_x_idx, h->d_x_xy, touched);
  // per-camera CSR of cross blocks for the implicit operator: code = 2 k + (camera is c1)
  std::vector<int> xptr(NC + 1, 0), xlist;
  {
    std::vector<std::vector<int>> per(NC);
    for (int k = 0; k < h->ncross; ++k) {
      per[cross_cam[k].x].push_back(2 * k);
      per[cross_cam[k].y].push_back(2 * k + 1);
    }
    for (int c = 0; c < NC; ++c) {
      xptr[c] = (int)xlist.size();
      xlist.insert(xlist.end(), per[c].begin(), per[c].end());
    }
    if (NC > 0) xptr[NC] = (int)xlist.size();
    h->nxlist = (int)xlist.size();
  }
  std::vector<int> chunk2_beg, seg2_chunk(NC + 1, 0), xcam_ptr(NC + 1, 0), xcam_list;
  int n2 = 0;
  int* sel2 = nullptr;
  if (h->pair_eval) {
    HIP_OK(hipMemsetAsync(small + 5, 0, sizeof(int) * 3, s));
    su_count_flags(s, NP, touched, small + 5);
    su_pair_intr(s, nx, h->d_x_idx, small + 7);
    // the entries that are not paired, per camera, in camera-major order
    unsigned char* uf = nullptr;
    int *ufi = nullptr, *uscan = nullptr, *iota = nullptr, *c2cnt_d = nullptr;
    CHECK_RC(tmp.alloc(&uf, std::max(1, NE)));
    CHECK_RC(tmp.alloc(&ufi, NE + 1));
    CHECK_RC(tmp.alloc(&uscan, NE + 1));
    CHECK_RC(tmp.alloc(&iota, std::max(1, NE)));
    CHECK_RC(tmp.alloc(&sel2, std::max(1, NE)));
    CHECK_RC(tmp.alloc(&c2cnt_d, NC + 1));
    su_unpaired_flags(s, NE, h->d_cm_idx, h->d_ext_col, uf, ufi);
    CHECK_RC(rp([&](void* t, size_t* b) { return su_exclusive_scan(t, b, ufi, uscan, NE + 1, s); }));
    su_gather_at(s, NC + 1, cam_cnt_d, uscan, c2cnt_d);
    su_iota(s, NE, iota);
    if (NE > 0)
      CHECK_RC(rp([&](void* t, size_t* b) { return su_select_flagged_i(t, b, iota, uf, sel2, small + 6, NE, s); }));
    std::vector<int> c2cnt(NC + 1, 0);
    CHECK_RC(d2h(c2cnt.data(), c2cnt_d, sizeof(int) * (NC + 1)));
    int pb[3] = {0, 0, 0};
    CHECK_RC(d2h(pb, small + 5, sizeof(int) * 3));
    HIP_OK(hipStreamSynchronize(s));
    h->pair_uni_intr = pb[2] == 0;
    h->pair_bytes = (16.0 + 12.0) * (double)nx + 24.0 * (double)pb[0] + 90.0 * 8.0 * h->nxchunk;
    n2 = pb[1];
    for (int c = 0; c < NC; ++c) {
      seg2_chunk[c] = (int)chunk2_beg.size();
      for (int q = c2cnt[c]; q < c2cnt[c + 1]; q += chunk) chunk2_beg.push_back(q);
    }
    seg2_chunk[NC] = (int)chunk2_beg.size();
    h->nchunk2 = (int)chunk2_beg.size();
    chunk2_beg.push_back(n2);
    std::vector<std::vector<int>> per(NC);
    for (int k = 0; k < h->ncross; ++k)
      for (int q = xseg_chunk[k]; q < xseg_chunk[k + 1]; ++q) {
        per[cross_cam[k].x].push_back(2 * q);
        per[cross_cam[k].y].push_back(2 * q + 1);
      }
    for (int c = 0; c < NC; ++c) {
      std::sort(per[c].begin(), per[c].end());
      xcam_ptr[c] = (int)xcam_list.size();
      xcam_list.insert(xcam_list.end(), per[c].begin(), per[c].end());
    }
    xcam_ptr[NC] = (int)xcam_list.size();
  }
  phase("device: pair-major");
  h->schur_built = false;
  h->schur_tiles = false;
  h->pcg_built = false;
  h->mf = h->mf32 = false;
  h->cg_wpart = nullptr;
  h->fused_grid = 0;
  h->mf_grid_n = 0;
  h->nblk = 0;
  h->nzero = 0;
  h->npairs = 0;

  // intrinsics: (cx, cy, fx, fy', k0, k1) with unused distortion terms zeroed
  std::vector<double> intr((size_t)kIntr * std::max(1, h->NI), 0.0);
  for (int i = 0; i < h->NI; ++i) {
    const double* K = p->intr + 6 * (size_t)i;
    double* o = &intr[(size_t)kIntr * i];
    o[0] = K[0];
    o[1] = K[1];
    o[2] = K[2];
    o[3] = p->intr_nf[i] == 2 ? K[3] : K[2];
    o[4] = p->intr_nk[i] >= 1 ? K[4] : 0.0;
    o[5] = p->intr_nk[i] >= 2 ? K[5] : 0.0;
  }
  std::vector<double> ext(p->ext, p->ext + 6 * (size_t)h->E);
  CHECK_RC(d.alloc(&h->d_arrivals, 1));
  HIP_OK(hipMemsetAsync(h->d_arrivals, 0, sizeof(unsigned), s));
  {
    std::vector<int> lists;
    for (int q = 0; q < nchunk; ++q)
      if (chunk_uni[q].x >= 0) lists.push_back(q);
    const int nuni = (int)lists.size();
    for (int q = 0; q < nchunk; ++q)
      if (chunk_uni[q].x < 0) lists.push_back(q);
    CHECK_RC(upload(&h->d_chunk_lists, d, lists, s));
    h->chunks.nchunk = nchunk;
    h->chunks.nuni = nuni;
    h->chunks.ngen = nchunk - nuni;
    h->chunks.uni = h->d_chunk_lists;
    h->chunks.gen = h->d_chunk_lists + nuni;
  }
  CHECK_RC(upload(&h->d_xchunk_beg, d, xchunk_beg, s));
  CHECK_RC(upload(&h->d_xseg_chunk, d, xseg_chunk, s));
  CHECK_RC(upload(&h->d_cross_cam, d, cross_cam, s));
  CHECK_RC(upload(&h->d_xptr, d, xptr, s));
  CHECK_RC(upload(&h->d_xlist, d, xlist, s));
  if (h->pair_eval) {
    if (n2 > 0) {
      CHECK_RC(d.alloc(&h->d_cm2_idx, (size_t)n2));
      CHECK_RC(d.alloc(&h->d_cm2_xy, (size_t)n2));
      su_gather_cm(s, n2, sel2, h->d_cm_idx, h->d_cm_xy, h->d_cm2_idx, h->d_cm2_xy);
    }
    CHECK_RC(upload(&h->d_chunk2_beg, d, chunk2_beg, s));
    CHECK_RC(upload(&h->d_seg2_chunk, d, seg2_chunk, s));
    CHECK_RC(upload(&h->d_xcam_ptr, d, xcam_ptr, s));
    if (!xcam_list.empty()) CHECK_RC(upload(&h->d_xcam_list, d, xcam_list, s));
    CHECK_RC(d.alloc(&h->d_partial2, (size_t)std::max(1, h->nchunk2) * 27));
    CHECK_RC(d.alloc(&h->d_xcpart, (size_t)h->nxchunk * 54));
  }
  CHECK_RC(upload(&h->d_intr, d, intr, s));
  CHECK_RC(d.alloc(&h->d_points, (size_t)3 * NP));
  su_points(s, NP, pt_of_d, r_points, h->d_points);
  CHECK_RC(upload(&h->d_ext, d, ext, s));
  h->host_entries = false;  // build_schur_* fetch the entry lists from the device on first use
  HIP_OK(hipStreamSynchronize(s));
  HIP_OK(hipGetLastError());
  phase("device: tables");
  return 0;
}

static int set_problem_impl(dab_handle* h, const dab_problem* p);
extern "C" int dab_set_problem(dab_handle* h, const dab_problem* p) {
  const int rc = set_problem_impl(h, p);
  CHECK_RC(guard_fail(h, "dab_set_problem"));
  return rc;
}
static int set_problem_impl(dab_handle* h, const dab_problem* p) {
  clear_error();
  if (!h) return set_error(DAB_E_INVALID, "null handle");
  CHECK_RC(validate(p));
  HIP_OK(hipSetDevice(h->device));
  HIP_OK(hipStreamSynchronize(h->stream));
  h->dev.release();
  // lazily allocated buffers went with the release: clear their pointers so that the next
  // use allocates again (a stale pointer would be written after its memory was freed)
  h->d_Yrec = nullptr;
  h->d_Y32c = h->d_Y32p = nullptr;
  h->d_Jfull = nullptr;
  h->have_problem = false;
  h->prob = *p;
  // DAB_SETUP_TIMING=1: phase times of the host preprocessing on stderr
  static const bool timing = getenv("DAB_SETUP_TIMING") != nullptr;
  double t_ph = now_s();
  auto phase = [&](const char* name) {
    if (!timing) return;
    const double t = now_s();
    fprintf(stderr, "set_problem %-22s %8.1f ms\n", name, 1e3 * (t - t_ph));
    t_ph = t;
  };
  const int N = p->num_obs;
  h->N = N;
  h->E = p->num_ext;
  h->NI = p->num_intr;

  const bool on_device = h->knobs.setup_host == 0 && setup_device_fits(h, p);
  if (on_device) CHECK_RC(setup_device(h, p, phase));
  else CHECK_RC(setup_host(h, p, phase));
  return setup_buffers(h, phase);
}


// Explicit-Schur tables (DAB_LINEAR_SOLVER_EXPLICIT_SCHUR only), built on first use:
// every ordered pair (e, f) of entries of one point with cam(e) >= cam(f) contributes
// -Y_e Y_f^T to lower block (cam(e), cam(f)) of the reduced camera system S. Pairs are
// sorted by block so each block is one deterministic segment. The block table is the
// union over ranks so the all-reduced packed layout matches.
static constexpr long long kMaxExplicitPairs = 200000000LL;
static int max_all_ranks(dab_handle* h, double& x) {  // max over ranks of one host scalar
  if (!h->coll()) return 0;
  hipStream_t s = h->stream;
  double* d_f = nullptr;
  CHECK_RC(h->dev.alloc(&d_f, 1));
  HIP_OK(hipMemcpyAsync(d_f, &x, sizeof(double), hipMemcpyHostToDevice, s));
  CHECK_RC(h->allreduce(d_f, 1, ncclMax));
  HIP_OK(hipMemcpyAsync(&x, d_f, sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  return 0;
}

// Explicit S by block tiles (k_schur_y + k_schur_tiles) when the camera set is small (the
// matrix-free criterion: tables in LDS, NC <= 160) and no point sees more than kTileMaxRec
// free cameras. Tables: each point's entries sorted by camera, records (distinct point-camera
// pairs), batches of whole points (<= 640 records, <= 64 points), tiles of <= 1024 blocks.
static constexpr int kBatchPts = 64, kTileBlocks = 1024;
// the entry lists on the host (the explicit-step table builders read them); the device
// set-up leaves them on the device until a builder asks
// The tile tables (k_schur_y / k_schur_tiles): per point its entries sorted by (camera,
// slot) (sch), one record per distinct (point, camera) ordered (batch, camera, point), batch
// headers, and the blocks' owners. On the device (dab_setup.hip, 19) unless the host entry
// lists are resident (DAB_SETUP_HOST=1: the host reference path); bitwise the same tables.
// d_sch / d_m: the device per-point sort (su_tile_sort) when on the device.
static int build_schur_tiles(dab_handle* h, int2* d_sch, const int* d_m) {
  hipStream_t s = h->stream;
  static const bool timing = getenv("DAB_SETUP_TIMING") != nullptr;
  double t_ph = now_s();
  auto phase = [&](const char* name) {
    if (!timing) return;
    const double t = now_s();
    fprintf(stderr, "schur_tiles %-22s %8.1f ms\n", name, 1e3 * (t - t_ph));
    t_ph = t;
  };
  const int NP = h->NP, NC = h->NC;
  const bool on_device = d_sch != nullptr;
  Dev& d = h->dev;
  const bool single = h->knobs.tile_single != 0;
  const int cap = schur_tile_batch_cap(NC, single);
  const int hdr_bytes = schur_tile_hdr_bytes(NC);
  const int nb = (int)tri_n(NC);
  std::vector<int> rec_ptr(NP + 1, 0);
  std::vector<int> batch_rec{0}, batch_pt{0};
  // batches of whole points: <= kBatchPts points (one mask word) and <= cap records
  auto cut_batches = [&]() {
    int cur = 0, curp = 0;
    for (int p = 0; p < NP; ++p) {
      const int m = rec_ptr[p + 1] - rec_ptr[p];
      if (curp > 0 && (cur + m > cap || curp + 1 > kBatchPts)) {
        batch_rec.push_back(rec_ptr[p]);
        batch_pt.push_back(p);
        cur = curp = 0;
      }
      cur += m;
      curp += 1;
    }
    batch_rec.push_back(rec_ptr[NP]);
    batch_pt.push_back(NP);
  };
  std::vector<long long> hits(std::max(1, nb), 0);
  int nbatch = 0, nrec = 0;
  int *d_br = nullptr, *d_bp = nullptr;
  unsigned char* d_hdr = nullptr;
  int4 *d_rec = nullptr, *d_robs = nullptr;
  if (on_device) {
    {
      std::vector<int> m(NP);
      if (NP > 0) HIP_OK(hipMemcpyAsync(m.data(), d_m, sizeof(int) * (size_t)NP, hipMemcpyDeviceToHost, s));
      HIP_OK(hipStreamSynchronize(s));
      for (int p = 0; p < NP; ++p) rec_ptr[p + 1] = rec_ptr[p] + m[p];
    }
    cut_batches();
    nbatch = (int)batch_rec.size() - 1;
    nrec = rec_ptr[NP];
    phase("device sort, batches");
    CHECK_RC(upload(&d_br, d, batch_rec, s));
    CHECK_RC(upload(&d_bp, d, batch_pt, s));
    CHECK_RC(d.alloc(&d_hdr, (size_t)std::max(1, nbatch) * hdr_bytes));
    CHECK_RC(d.alloc(&d_rec, (size_t)std::max(1, nrec)));
    CHECK_RC(d.alloc(&d_robs, (size_t)std::max(1, nrec)));
    HIP_OK(hipMemsetAsync(d_hdr, 0, (size_t)std::max(1, nbatch) * hdr_bytes, s));
    su_tile_batch(s, nbatch, NC, d_bp, d_br, h->d_pt_ent_ptr, d_sch, h->d_obs_idx, hdr_bytes, d_hdr, d_rec, d_robs);
    int* d_hits = nullptr;
    CHECK_RC(h->setup_tmp.alloc(&d_hits, (size_t)std::max(1, nb)));
    HIP_OK(hipMemsetAsync(d_hits, 0, sizeof(int) * (size_t)std::max(1, nb), s));
    su_tile_hits(s, NP, nb, h->d_pt_ent_ptr, d_sch, d_hits);
    std::vector<int> hi(std::max(1, nb));
    HIP_OK(hipMemcpyAsync(hi.data(), d_hits, sizeof(int) * (size_t)std::max(1, nb), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    for (int k = 0; k < nb; ++k) hits[k] = hi[k];
    phase("device records, hits");
  } else {
    const std::vector<int>& pt_ent_ptr = h->h_pt_ent_ptr;
    const big_vec<int>& ent_cam = h->h_ent_cam;
    const big_vec<int>& ent_os = h->h_ent_os;
    big_vec<int2> sch(h->NE);
    // per point (threads): entries sorted by (camera, slot), distinct cameras counted
    par_for(NP, [&](long long pb, long long pe, int) {
      for (int p = (int)pb; p < (int)pe; ++p) {
        const int b = pt_ent_ptr[p], e = pt_ent_ptr[p + 1];
        for (int i = b; i < e; ++i) sch[i] = make_int2(ent_os[i], ent_cam[i]);
        std::sort(sch.begin() + b, sch.begin() + e, [](const int2& x, const int2& y) {
          return x.y != y.y ? x.y < y.y : x.x < y.x;
        });
        int m = 0;
        for (int i = b; i < e; ++i) m += (i == b || sch[i].y != sch[i - 1].y);
        rec_ptr[p + 1] = m;
      }
    }, 2048);
    for (int p = 0; p < NP; ++p) rec_ptr[p + 1] += rec_ptr[p];
    nrec = rec_ptr[NP];
    phase("sort entries");
    cut_batches();
    nbatch = (int)batch_rec.size() - 1;
    // records ordered (batch, camera, point) and the batch headers: mask[NC] | off[NC + 1]
    big_vec<int4> rec(nrec), robs(nrec);
    std::vector<unsigned char> hdr((size_t)nbatch * hdr_bytes, 0);
    par_for(nbatch, [&](long long bb, long long be, int) {
      std::vector<int> pos(NC + 1);
      for (int b = (int)bb; b < (int)be; ++b) {
        unsigned long long* mask = reinterpret_cast<unsigned long long*>(&hdr[(size_t)b * hdr_bytes]);
        int* off = reinterpret_cast<int*>(&hdr[(size_t)b * hdr_bytes + 8 * (size_t)NC]);
        for (int p = batch_pt[b]; p < batch_pt[b + 1]; ++p)
          for (int i = pt_ent_ptr[p]; i < pt_ent_ptr[p + 1]; ++i)
            if (i == pt_ent_ptr[p] || sch[i].y != sch[i - 1].y) {
              off[sch[i].y + 1]++;
              mask[sch[i].y] |= 1ull << (p - batch_pt[b]);
            }
        for (int c = 0; c < NC; ++c) off[c + 1] += off[c];
        for (int c = 0; c <= NC; ++c) pos[c] = off[c];
        for (int p = batch_pt[b]; p < batch_pt[b + 1]; ++p) {
          int r = -1;
          for (int i = pt_ent_ptr[p]; i < pt_ent_ptr[p + 1]; ++i) {
            if (i > pt_ent_ptr[p] && sch[i].y == sch[i - 1].y) {
              rec[r].y++;
              continue;
            }
            r = batch_rec[b] + pos[sch[i].y]++;
            rec[r] = make_int4(i, 1, p, sch[i].y);
            const int o = h->perm[sch[i].x >> 1];  // the caller's observation of the slot
            robs[r] = make_int4(sch[i].x, h->prob.obs_ext0[o], h->prob.obs_ext1[o], h->prob.obs_intr[o]);
          }
        }
      }
    }, 16);
    phase("records, headers");
    // hit counts of every block from a sample of the points (every 4th): the points that see
    // both of its cameras
    std::vector<std::vector<long long>> th(setup_threads(), std::vector<long long>(std::max(1, nb), 0));
    par_for(NP, [&](long long pb, long long pe, int t) {
      std::vector<int> cams;
      for (int p = (int)pb; p < (int)pe; ++p) {
        if (p % 4) continue;
        cams.clear();
        for (int i = pt_ent_ptr[p]; i < pt_ent_ptr[p + 1]; ++i)
          if (i == pt_ent_ptr[p] || sch[i].y != sch[i - 1].y) cams.push_back(sch[i].y);
        for (size_t x = 0; x < cams.size(); ++x)  // ascending: block (cams[x], cams[y <= x])
          for (size_t y = 0; y <= x; ++y) th[t][tri_n(cams[x]) + cams[y]]++;
      }
    });
    for (auto& v : th)
      for (int k = 0; k < nb; ++k) hits[k] += v[k];
    CHECK_RC(upload(&d_br, d, batch_rec, s));
    CHECK_RC(upload(&d_hdr, d, hdr, s));
    CHECK_RC(upload(&d_sch, d, sch, s));
    CHECK_RC(upload(&d_rec, d, rec, s));
    CHECK_RC(upload(&d_robs, d, robs, s));
    phase("hits, upload");
  }
  // tiles: equal block ranges of <= kTileBlocks (rows up to the tile's last camera)
  const int ntile = std::max(1, (nb + kTileBlocks - 1) / kTileBlocks);
  std::vector<int> tb(ntile + 1), clast(ntile);
  for (int t = 0; t <= ntile; ++t) tb[t] = (int)((long long)nb * t / ntile);
  // slots: per tile, blocks by hit count (descending); thread i owns the i-th heaviest and
  // the (1023 - i)-th, so the pairs' sums are even and a wave's threads have similar work
  std::vector<int> slot((size_t)ntile * 2 * kTileThreads, -1);
  for (int t = 0; t < ntile; ++t) {
    std::vector<int> bl;
    for (int k = tb[t]; k < tb[t + 1]; ++k) bl.push_back(k);
    std::stable_sort(bl.begin(), bl.end(), [&](int x, int y) { return hits[x] > hits[y]; });
    for (int i = 0; i < (int)bl.size(); ++i) {
      const int th2 = i < kTileThreads ? i : 2 * kTileThreads - 1 - i;
      slot[(size_t)t * 2 * kTileThreads + (i < kTileThreads ? 0 : kTileThreads) + th2] = bl[i];
    }
    int c = 0;
    while (tri_n(c + 1) <= tb[t + 1] - 1) ++c;
    clast[t] = c;
  }
  phase("slots");
  SchurTiles& a = h->tiles;
  a.ntile = ntile;
  a.nbatch = nbatch;
  a.nrec = nrec;
  // load balance: a tile's time is its busiest wave's, summed over its batches, and the
  // tiles differ (C5: the arc rows' tile ~2x the others), so a heavy tile's batches go to
  // several work-groups per group. Parts per tile from the sampled hits (the tile's work):
  // the split that minimises max_t(hits_t / sub_t) / groups, groups = CUs / sum(sub)
  // (multiples of 8: one XCD per group). DAB_TILE_BALANCE=0 keeps one part per tile.
  std::vector<int> sub(ntile, 1);
  {
    std::vector<double> w(ntile, 0.0);
    for (int t = 0; t < ntile; ++t)
      for (int k = tb[t]; k < tb[t + 1]; ++k) w[t] += (double)hits[k] + 1.0;
    auto groups_for = [&](int nsub) {
      int ng = std::max(1, h->ncu / nsub);
      if (ng >= 8) ng -= ng % 8;
      return ng;
    };
    auto cost = [&](const std::vector<int>& sb) {
      int ns = 0;
      double m = 0.0;
      for (int t = 0; t < ntile; ++t) {
        ns += sb[t];
        m = std::max(m, w[t] / sb[t]);
      }
      return m / groups_for(ns);
    };
    if (h->knobs.tile_balance != 0 && ntile > 1 && ntile <= 6) {
      std::vector<int> cur(ntile, 1), best = cur;
      double bc = cost(cur);
      for (;;) {  // odometer over sub_t in 1..4
        int t = 0;
        while (t < ntile && cur[t] == 4) cur[t++] = 1;
        if (t == ntile) break;
        ++cur[t];
        const double c = cost(cur);
        if (c < bc * (1.0 - 1e-12)) {
          bc = c;
          best = cur;
        }
      }
      sub = best;
    }
  }
  std::vector<int> subbeg(ntile + 1, 0);
  for (int t = 0; t < ntile; ++t) subbeg[t + 1] = subbeg[t] + sub[t];
  a.nsub = subbeg[ntile];
  int ng = std::max(1, h->ncu / a.nsub);
  if (ng >= 8) ng -= ng % 8;
  // at least tile_minb batches per work-group (small problems keep few partials for the sum):
  // 2 since round 6 — C1's 313 batches on 156 work-groups instead of 39, k_schur_tiles
  // 153 -> 57 us, its partial sum 7 -> 15 us (scripts/runs/r06h.sh)
  const int smax = *std::max_element(sub.begin(), sub.end());
  a.ngroup = std::max(1, std::min(ng, a.nbatch / (std::max(1, h->knobs.tile_minb) * smax)));
  std::vector<int> blk_nslot(std::max(1, nb), a.ngroup);
  for (int t = 0; t < ntile; ++t)
    for (int k = tb[t]; k < tb[t + 1]; ++k) blk_nslot[k] = a.ngroup * sub[t];
  a.nelem = 36 * nb;
  a.stride = (size_t)a.nelem;
  a.kq = 0;
  a.batch_cap = cap;
  a.single = single ? 1 : 0;
  a.hdr_bytes = hdr_bytes;
  int *d_cl = nullptr, *d_slot = nullptr;
  CHECK_RC(upload(&d_cl, d, clast, s));
  CHECK_RC(upload(&d_slot, d, slot, s));
  a.rec_obs = d_robs;
  a.batch_rec = d_br;
  a.tile_clast = d_cl;
  a.tile_slot = d_slot;
  a.hdr = d_hdr;
  a.sch_ent = d_sch;
  a.rec_info = d_rec;
  CHECK_RC(d.alloc(&h->d_kx, (size_t)6 * NC));
  a.kx = h->d_kx;
  CHECK_RC(d.alloc(&a.partial, (size_t)a.ngroup * smax * a.stride));
  int *d_sub = nullptr, *d_subbeg = nullptr, *d_nslot = nullptr;
  CHECK_RC(upload(&d_sub, d, sub, s));
  CHECK_RC(upload(&d_subbeg, d, subbeg, s));
  CHECK_RC(upload(&d_nslot, d, blk_nslot, s));
  a.tile_sub = d_sub;
  a.tile_subbeg = d_subbeg;
  a.blk_nslot = d_nslot;
  CHECK_RC(d.alloc(&h->d_sblk, a.stride));
  CHECK_RC(d.alloc(&h->d_rfx, (size_t)6 * NC));
  CHECK_RC(d.alloc(&h->d_yrec, (size_t)18 * std::max(1, a.nrec)));
  HIP_OK(hipStreamSynchronize(s));
  phase("upload, alloc");
  return 0;
}

// present block keys: the union over ranks (every rank must all-reduce the same S layout)
static int union_block_keys(dab_handle* h, std::vector<long long>& keys) {
  if (!h->coll()) return 0;
  const int NC = h->NC;
  hipStream_t s = h->stream;
  std::vector<double> bm((size_t)NC * NC, 0.0);
  for (long long k : keys) bm[(size_t)k] = 1.0;
  double* d_bm = nullptr;
  CHECK_RC(h->dev.alloc(&d_bm, bm.size()));
  HIP_OK(hipMemcpyAsync(d_bm, bm.data(), bm.size() * sizeof(double), hipMemcpyHostToDevice, s));
  CHECK_RC(h->allreduce(d_bm, bm.size(), ncclMax));
  HIP_OK(hipMemcpyAsync(bm.data(), d_bm, bm.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  keys.clear();
  for (size_t i = 0; i < bm.size(); ++i)
    if (bm[i] != 0.0) keys.push_back((long long)i);
  return 0;
}

// Pair tables on the device (dab_setup.hip, 18): h->d_pairs in sorted (key, e, f) order;
// pk / pbeg: the present keys (increasing) and their first pair; np2 pairs
static int build_schur_pairs_device(dab_handle* h, std::vector<long long>& pk, std::vector<int>& pbeg,
                                    long long& np2) {
  hipStream_t s = h->stream;
  const int NP = h->NP, NC = h->NC;
  // block key c0 * NC + c1 is a 32-bit int (a dense S that large would not fit anyway)
  if ((long long)NC * NC > (long long)INT_MAX)
    return set_error(DAB_E_UNSUPPORTED, "explicit Schur pair tables for more than 46340 free cameras");
  Dev& tmp = h->setup_tmp;  // released at the next set-up
  void* rtmp = nullptr;
  size_t rtmp_cap = 0;
  auto rp = [&](auto call) -> int {
    size_t bytes = 0;
    if (call(nullptr, &bytes) != 0) return set_error(DAB_E_DEVICE, "rocPRIM size query failed");
    if (bytes > rtmp_cap) {
      void* q = nullptr;
      CHECK_RC(tmp.alloc(reinterpret_cast<unsigned char**>(&q), bytes));
      rtmp = q;
      rtmp_cap = bytes;
    }
    if (call(rtmp, &bytes) != 0) return set_error(DAB_E_DEVICE, "rocPRIM pass failed");
    return 0;
  };
  int* cnt = nullptr;
  unsigned long long* tot = nullptr;
  CHECK_RC(tmp.alloc(&cnt, (size_t)NP + 1));
  CHECK_RC(tmp.alloc(&tot, 1));
  HIP_OK(hipMemsetAsync(tot, 0, sizeof(unsigned long long), s));
  HIP_OK(hipMemsetAsync(cnt + NP, 0, sizeof(int), s));
  su_pair_count(s, NP, h->d_pt_ent_ptr, h->d_ent_cam, cnt, tot);
  unsigned long long total = 0;
  HIP_OK(hipMemcpyAsync(&total, tot, sizeof(total), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  double flag = NC > 0 && (long long)total > kMaxExplicitPairs ? 1.0 : 0.0;
  CHECK_RC(max_all_ranks(h, flag));  // every rank must take the same branch
  if (flag != 0.0)
    return set_error(DAB_E_UNSUPPORTED,
                     "reduced camera system too large for explicit Schur pair tables (" + std::to_string(total) +
                         " pairs); use DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG");
  np2 = NC > 0 ? (long long)total : 0;
  const int n = (int)np2;
  pk.clear();
  pbeg.clear();
  CHECK_RC(h->dev.alloc(&h->d_pairs, (size_t)std::max(1, n)));
  if (n == 0) return 0;
  int *poff = nullptr, *k1 = nullptr, *v1 = nullptr, *k2 = nullptr, *v2 = nullptr, *uk = nullptr, *uc = nullptr,
      *nr = nullptr;
  int2* ef = nullptr;
  CHECK_RC(tmp.alloc(&poff, (size_t)NP + 1));
  CHECK_RC(tmp.alloc(&k1, (size_t)n));
  CHECK_RC(tmp.alloc(&v1, (size_t)n));
  CHECK_RC(tmp.alloc(&k2, (size_t)n));
  CHECK_RC(tmp.alloc(&v2, (size_t)n));
  CHECK_RC(tmp.alloc(&ef, (size_t)n));
  CHECK_RC(rp([&](void* t, size_t* b) { return su_exclusive_scan(t, b, cnt, poff, NP + 1, s); }));
  su_pair_gen(s, NP, h->d_pt_ent_ptr, h->d_ent_cam, poff, NC, k1, v1, ef);
  CHECK_RC(rp([&](void* t, size_t* b) { return su_sort_pairs(t, b, k1, k2, v1, v2, n, bits_for(NC * NC), s); }));
  su_pair_gather(s, n, v2, ef, h->d_ent_pos, h->d_pairs);
  // present keys and their run lengths
  uk = k1;  // the unsorted keys are no longer needed
  uc = v1;
  CHECK_RC(tmp.alloc(&nr, 1));
  CHECK_RC(rp([&](void* t, size_t* b) { return su_rle(t, b, k2, uk, uc, nr, n, s); }));
  int nruns = 0;
  HIP_OK(hipMemcpyAsync(&nruns, nr, sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  std::vector<int> ukh(nruns), uch(nruns);
  HIP_OK(hipMemcpyAsync(ukh.data(), uk, sizeof(int) * (size_t)nruns, hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(uch.data(), uc, sizeof(int) * (size_t)nruns, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  pk.resize(nruns);
  pbeg.resize(nruns);
  int acc = 0;
  for (int i = 0; i < nruns; ++i) {
    pk[i] = ukh[i];
    pbeg[i] = acc;
    acc += uch[i];
  }
  return 0;
}

static int build_schur_tables(dab_handle* h) {
  if (h->schur_built) return 0;
  static const bool timing = getenv("DAB_SETUP_TIMING") != nullptr;
  const double t_b = now_s();
  struct Report {
    bool on;
    double t0;
    ~Report() {
      if (on) fprintf(stderr, "build_schur_tables %8.1f ms\n", 1e3 * (now_s() - t0));
    }
  } report{timing, t_b};
  double t_ph = t_b;
  auto phase = [&](const char* name) {
    if (!timing) return;
    const double t = now_s();
    fprintf(stderr, "schur_tables %-21s %8.1f ms\n", name, 1e3 * (t - t_ph));
    t_ph = t;
  };
  hipStream_t s = h->stream;
  const int NP = h->NP, NC = h->NC;
  const std::vector<int>& pt_ent_ptr = h->h_pt_ent_ptr;
  const big_vec<int>& ent_cam = h->h_ent_cam;
  const big_vec<int>& ent_pos = h->h_ent_pos;
  int2* tile_sch = nullptr;
  int* tile_m = nullptr;
  int dev_maxm = 0;
  {
    // tile mode: every rank must take the same branch (the all-reduced S layouts differ).
    // The host entry lists are needed by the tile tables (and by the host reference path of
    // the pair tables); large camera sets with device set-up never fetch them.
    const bool tiles_possible = h->knobs.schur_tiles != 0 && NC > 0 && mf_schur_fits(NC, h->E, h->NI);
    if (tiles_possible && !h->host_entries) {
      // device: per point entries sorted by (camera, slot), distinct cameras counted
      CHECK_RC(h->dev.alloc(&tile_sch, (size_t)std::max(1, h->NE)));
      CHECK_RC(h->setup_tmp.alloc(&tile_m, (size_t)std::max(1, NP)));
      su_tile_sort(s, NP, h->d_pt_ent_ptr, h->d_ent_cam, h->d_ent_os, tile_sch, tile_m);
      if (NP > 0) {
        int* d_max = nullptr;
        CHECK_RC(h->setup_tmp.alloc(&d_max, 1));
        size_t bytes = 0;
        if (su_max(nullptr, &bytes, tile_m, d_max, NP, s) != 0) return set_error(DAB_E_DEVICE, "rocPRIM size query failed");
        unsigned char* t = nullptr;
        CHECK_RC(h->setup_tmp.alloc(&t, std::max<size_t>(1, bytes)));
        if (su_max(t, &bytes, tile_m, d_max, NP, s) != 0) return set_error(DAB_E_DEVICE, "rocPRIM pass failed");
        HIP_OK(hipMemcpyAsync(&dev_maxm, d_max, sizeof(int), hipMemcpyDeviceToHost, s));
        HIP_OK(hipStreamSynchronize(s));
      }
    }
    std::vector<int> tmax(setup_threads(), 0);  // distinct free cameras of one point
    if (tiles_possible && h->host_entries) par_for(NP, [&](long long pb, long long pe, int t) {
      std::vector<int> seen(std::max(1, NC), -1);
      for (int pt = (int)pb; pt < (int)pe; ++pt) {
        int m = 0;
        for (int e = pt_ent_ptr[pt]; e < pt_ent_ptr[pt + 1]; ++e)
          if (seen[ent_cam[e]] != pt) {
            seen[ent_cam[e]] = pt;
            ++m;
          }
        tmax[t] = std::max(tmax[t], m);
      }
    });
    const int maxm = std::max(dev_maxm, *std::max_element(tmax.begin(), tmax.end()));
    phase("camera counts");
    double no_tiles = (tiles_possible && maxm <= kTileMaxRec) ? 0.0 : 1.0;
    CHECK_RC(max_all_ranks(h, no_tiles));
    h->schur_tiles = no_tiles == 0.0;
  }
  if (h->schur_tiles) {
    CHECK_RC(build_schur_tiles(h, tile_sch, tile_m));
    t_ph = now_s();
    h->nblk = 0;
    h->nzero = 0;
    h->npairs = 0;
    CHECK_RC(h->dev.alloc(&h->d_spack, h->spack_count()));  // ybc only
    phase("tiles: spack alloc");
    const int n = 6 * NC;
    h->lds = ((n + 1 + 7) / 8) * 8;
    if (h->lds % 512 == 0) h->lds += 8;
    CHECK_RC(h->sticky(h->st_S, &h->d_S, (size_t)(n + 1) * h->lds));
    h->mf_grid_n = mf_grid(h->NP, h->ncu);
    phase("tiles: S alloc");
    h->schur_built = true;
    return 0;
  }
  // reduced-camera-system blocks: ordered entry pairs (e, f) of one point with
  // cam(e) >= cam(f); block (cam(e), cam(f)) of the lower triangle of S.
  std::vector<long long> blkkeys;
  std::vector<int2> pairs;
  std::vector<int> blk_pair_beg;
  const bool on_device = !h->host_entries;
  if (on_device) {
    // device: count, scan, generate, stable radix sort by block key, gather (bitwise the
    // host path's tables; the pairs stay on the device)
    std::vector<long long> pk;
    std::vector<int> pbeg;
    long long np2 = 0;
    CHECK_RC(build_schur_pairs_device(h, pk, pbeg, np2));
    phase("pairs on device");
    std::vector<long long> diag((size_t)NC), keys;
    for (int c = 0; c < NC; ++c) diag[c] = (long long)c * NC + c;
    keys.reserve(pk.size() + diag.size());
    std::merge(pk.begin(), pk.end(), diag.begin(), diag.end(), std::back_inserter(keys));
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    CHECK_RC(union_block_keys(h, keys));
    blkkeys = keys;
    blk_pair_beg.assign(blkkeys.size() + 1, 0);
    size_t j = 0;
    for (size_t b2 = 0; b2 < blkkeys.size(); ++b2) {
      while (j < pk.size() && pk[j] < blkkeys[b2]) ++j;
      blk_pair_beg[b2] = j < pk.size() ? pbeg[j] : (int)np2;
    }
    blk_pair_beg[blkkeys.size()] = (int)np2;
    h->npairs = np2;
  }
  long long total = 0;
  if (!on_device) {
    for (int pt = 0; pt < NP; ++pt) {
      const long long m = pt_ent_ptr[pt + 1] - pt_ent_ptr[pt];
      total += m * (m + 1) / 2 + m;  // upper bound
    }
    double flag = total > kMaxExplicitPairs ? 1.0 : 0.0;
    CHECK_RC(max_all_ranks(h, flag));  // every rank must take the same branch
    if (flag != 0.0)
      return set_error(DAB_E_UNSUPPORTED,
                       "reduced camera system too large for explicit Schur pair tables (" +
                           std::to_string(total) + " pairs); use DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG");
  }
  if (on_device) {
  } else if (NC > 0) {
    // pairs generated per point in parallel, in (e, f) order (entries are point-major, so
    // that is the global (e, f) order), then a stable counting sort by block key: the
    // (key, e, f) order of the former comparison sort (~0.4 s at C3), bitwise the same tables
    std::vector<long long> poff((size_t)NP + 1, 0);
    par_for(NP, [&](long long pb, long long pe, int) {
      for (int pt = (int)pb; pt < (int)pe; ++pt) {
        long long c = 0;
        for (int e = pt_ent_ptr[pt]; e < pt_ent_ptr[pt + 1]; ++e)
          for (int f = pt_ent_ptr[pt]; f < pt_ent_ptr[pt + 1]; ++f) c += ent_cam[e] >= ent_cam[f];
        poff[pt + 1] = c;
      }
    }, 4096);
    for (int pt = 0; pt < NP; ++pt) poff[pt + 1] += poff[pt];
    const long long np2 = poff[NP];
    big_vec<long long> pkey((size_t)np2);  // c0 * NC + c1 in 64 bits
    big_vec<int2> pef((size_t)np2);
    par_for(NP, [&](long long pb, long long pe, int) {
      for (int pt = (int)pb; pt < (int)pe; ++pt) {
        long long o = poff[pt];
        for (int e = pt_ent_ptr[pt]; e < pt_ent_ptr[pt + 1]; ++e)
          for (int f = pt_ent_ptr[pt]; f < pt_ent_ptr[pt + 1]; ++f) {
            const int ce = ent_cam[e], cf = ent_cam[f];
            if (ce < cf) continue;
            pkey[o] = (long long)ce * NC + cf;
            pef[o] = make_int2(e, f);
            ++o;
          }
      }
    }, 4096);
    // two stable counting passes (by cf, then by ce: memory O(threads x NC), not NC^2)
    phase("pairs generated");
    big_vec<int> o1, o2;
    std::vector<long long> st1, st2;
    bucket_sort(np2, NC, [&](long long i) { return (int)(pkey[i] % NC); }, o1, st1);
    bucket_sort(np2, NC, [&](long long j) { return (int)(pkey[o1[j]] / NC); }, o2, st2);
    pairs.resize((size_t)np2);
    big_vec<long long> skey((size_t)np2);
    par_for(np2, [&](long long pb, long long pe, int) {
      for (long long i = pb; i < pe; ++i) {
        const int q = o1[o2[i]];
        const int2 ef = pef[q];
        pairs[i] = make_int2(ent_pos[ef.x], ent_pos[ef.y]);  // Y records are camera-major
        skey[i] = pkey[q];
      }
    });
    phase("pairs sorted");
    // present keys with their first pair, in increasing key order
    std::vector<long long> pk;
    std::vector<int> pbeg;
    pk.reserve((size_t)NC * 64);
    pbeg.reserve((size_t)NC * 64);
    for (long long i = 0; i < np2; ++i)
      if (i == 0 || skey[i] != skey[i - 1]) {
        pk.push_back(skey[i]);
        pbeg.push_back((int)i);
      }
    // diagonal blocks always exist; union across ranks
    std::vector<long long> diag((size_t)NC), keys;
    for (int c = 0; c < NC; ++c) diag[c] = (long long)c * NC + c;
    keys.reserve(pk.size() + diag.size());
    std::merge(pk.begin(), pk.end(), diag.begin(), diag.end(), std::back_inserter(keys));  // both sorted
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    CHECK_RC(union_block_keys(h, keys));
    blkkeys = keys;
    blk_pair_beg.assign(blkkeys.size() + 1, 0);
    size_t j = 0;  // blocks without local pairs start where the next present key does
    for (size_t b2 = 0; b2 < blkkeys.size(); ++b2) {
      while (j < pk.size() && pk[j] < blkkeys[b2]) ++j;
      blk_pair_beg[b2] = j < pk.size() ? pbeg[j] : (int)np2;
    }
    blk_pair_beg[blkkeys.size()] = (int)np2;
  } else {
    blk_pair_beg.assign(1, 0);
  }
  phase("block keys");
  h->nblk = (int)blkkeys.size();
  if (!on_device) h->npairs = (long long)pairs.size();
  std::vector<int2> blk_cam(h->nblk);
  for (int b = 0; b < h->nblk; ++b) blk_cam[b] = make_int2((int)(blkkeys[b] / NC), (int)(blkkeys[b] % NC));

  // the lower blocks no pair reaches (blkkeys is sorted): zeroed per step on one rank, where
  // the blocks are written into S directly
  std::vector<int2> blk_zero;
  {
    size_t j = 0;
    for (int c = 0; c < NC; ++c)
      for (int d2 = 0; d2 <= c; ++d2) {
        const long long key = (long long)c * NC + d2;
        while (j < blkkeys.size() && blkkeys[j] < key) ++j;
        if (j >= blkkeys.size() || blkkeys[j] != key) blk_zero.push_back(make_int2(c, d2));
      }
  }
  h->nzero = (int)blk_zero.size();

  Dev& d = h->dev;
  if (!on_device) CHECK_RC(upload(&h->d_pairs, d, pairs, s));
  CHECK_RC(upload(&h->d_blk_cam, d, blk_cam, s));
  if (h->nzero > 0) CHECK_RC(upload(&h->d_blk_zero, d, blk_zero, s));
  CHECK_RC(upload(&h->d_blk_pair_beg, d, blk_pair_beg, s));
  CHECK_RC(d.alloc(&h->d_spack, h->spack_count()));
  const int n = 6 * NC;
  h->lds = ((n + 1 + 7) / 8) * 8;
  if (h->lds % 512 == 0) h->lds += 8;  // avoid power-of-two row strides
  CHECK_RC(h->sticky(h->st_S, &h->d_S, NC > 0 ? (size_t)(n + 1) * h->lds : 1));
  // Y as [NE][18] records for k_s_blocks (allocated here so that an OOM surfaces before
  // iteration 0, not mid-solve)
  if (NC > 0) CHECK_RC(d.alloc(&h->d_Yrec, (size_t)kYRec * std::max(1, h->NE)));
  HIP_OK(hipStreamSynchronize(s));
  phase("upload, alloc");
  h->schur_built = true;
  return 0;
}

// Implicit-Schur PCG buffers (DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG), allocated on first use.
static int build_pcg_buffers(dab_handle* h) {
  if (h->pcg_built) return 0;
  Dev& d = h->dev;
  const size_t n = (size_t)6 * h->NC;
  for (double** b : {&h->d_pcg_b, &h->d_pcg_r, &h->d_pcg_z, &h->d_pcg_p, &h->d_pcg_q, &h->d_pcg_w})
    CHECK_RC(d.alloc(b, n));
  CHECK_RC(d.alloc(&h->d_pcg_Ad, 6 * n));
  CHECK_RC(d.alloc(&h->d_pcg_Minv, 6 * n));
  CHECK_RC(d.alloc(&h->d_pcg_red, (size_t)27 * h->NC));
  CHECK_RC(d.alloc(&h->d_pcg_t, (size_t)4 * h->NP));
  CHECK_RC(d.alloc(&h->d_pcg_state, 1));
  CHECK_RC(d.alloc(&h->d_cg_partial, (size_t)cg_partial_size(h->NC)));
  CHECK_RC(d.alloc(&h->d_cg_cnt, 1));
  HIP_OK(hipMemsetAsync(h->d_cg_cnt, 0, sizeof(unsigned), h->stream));
  // the single-pass matvec when the camera system is small (DAB_PCG_FUSED=0 disables it)
  h->mf = mf_schur_fits(h->NC, h->E, h->NI) && h->NP > 0 && h->knobs.pcg_mf != 0;
  if (h->mf) {
    h->mf_grid_n = mf_grid(h->NP, h->ncu);
    CHECK_RC(d.alloc(&h->d_mf_partial, (size_t)h->mf_grid_n * 6 * h->NC));
  }
  h->fused_grid = 0;
  if (pcg_fused_fits(h->NC) && h->NP > 0 && h->knobs.pcg_fused != 0) {
    h->fused_grid = pcg_fused_grid(h->NP, h->ncu);
    CHECK_RC(d.alloc(&h->d_fused_partial, (size_t)h->fused_grid * 6 * h->NC));
  }
  if (!h->h_pcg_state && !(h->h_pcg_state = static_cast<PcgState*>(pinned_take(sizeof(PcgState)))))
    return set_error(DAB_E_NOMEM, "pinned PCG state allocation failed");
  h->pcg_built = true;
  return 0;
}

// S vec (Y part) -> d_pcg_w, all-reduced across ranks
// exact: the fp64 product even in a mixed-precision solve (the true residual r = b - S x)
static int pcg_matvec(dab_handle* h, YBufs yb, const double* vec, bool exact = false) {
  hipStream_t s = h->stream;
  // the stored-Y products all-reduce into d_pcg_w; only the one-rank matrix-free product
  // hands its work-group partials to the CG update (never left over from an earlier problem)
  h->cg_wpart = nullptr;
  if (h->mf) {
    // one rank with cross blocks (the rig): the product's partials are summed inside the CG
    // update (no all-reduce in between), one launch fewer per iteration. A one-rank RCCL
    // handle takes this path too (its all-reduce of a single rank is the identity, and the
    // separate partial-sum launch would regroup the sums: the trajectory would leave
    // dab_create's in the last bits)
    const bool fuse = h->world == 1 && h->nxlist > 0 && h->knobs.cg_onewg == 0;
    h->cg_wpart = fuse ? h->d_mf_partial : nullptr;
    double* w = fuse ? nullptr : h->d_pcg_w;
    if (h->mf32 && !exact)
      launch_mf_product32(s, h->view, h->d_points, h->d_camtab, h->d_scale_c, h->d_L, vec, h->d_mf_partial, w,
                          h->mf_grid_n, h->d_pcg_state);
    else
      launch_mf_product(s, h->view, h->d_points, h->d_camtab, h->d_scale_c, h->d_L, vec, h->d_mf_partial, w,
                        h->mf_grid_n, h->d_pcg_state);
    if (!fuse) CHECK_RC(h->allreduce(h->d_pcg_w, (size_t)6 * h->NC, ncclSum));
    return 0;
  }
  if (h->fused_grid > 0) {
    launch_pcg_fused(s, h->view, yb, vec, h->d_fused_partial, h->d_pcg_w, h->fused_grid, h->d_pcg_state);
    CHECK_RC(h->allreduce(h->d_pcg_w, (size_t)6 * h->NC, ncclSum));
    return 0;
  }
  const bool direct = h->nchunk == h->NC;
  launch_pcg_matvec_passes(s, h->view, h->nchunk, h->d_chunk_beg, yb, vec, h->d_pcg_t,
                           direct ? h->d_pcg_w : h->d_partial, h->d_pcg_state);
  if (!direct) launch_seg_final(s, h->NC, 6, h->d_seg_chunk, h->d_partial, h->d_pcg_w, h->max_seg_chunks);
  CHECK_RC(h->allreduce(h->d_pcg_w, (size_t)6 * h->NC, ncclSum));
  return 0;
}

// Solve S y = b (scaled, damped reduced camera system) into d_yc with preconditioned CG.
// Requires d_L, d_q (point factor) and d_Y (entry_y) of this step. Returns the number of
// CG iterations in *iters and the final PcgState status in *status.
static int pcg_solve(dab_handle* h, const dab_options& opt, StepScalars sc, YBufs yb, int* iters, int* status) {
  hipStream_t s = h->stream;
  const DevView& v = h->view;
  const int NC = h->NC;
  const bool direct = h->nchunk == h->NC;
  if (h->mf)
    launch_mf_diag_rhs(s, v, h->nchunk, h->d_run_beg, h->d_run_rec, h->d_points, h->d_camtab, h->d_scale_c, h->d_L,
                       h->d_q, direct ? h->d_pcg_red : h->d_partial);
  else
    launch_pcg_diag_rhs_partial(s, v, h->nchunk, h->d_chunk_beg, h->d_run, yb, h->d_q,
                                direct ? h->d_pcg_red : h->d_partial);
  if (!direct) launch_seg_final(s, NC, 27, h->d_seg_chunk, h->d_partial, h->d_pcg_red, h->max_seg_chunks);
  CHECK_RC(h->allreduce(h->d_pcg_red, (size_t)27 * NC, ncclSum));
  launch_pcg_setup(s, NC, h->ug(), h->d_scale_c, sc, h->d_pcg_red, h->d_pcg_Ad, h->d_pcg_Minv, h->d_pcg_b,
                   h->d_yc, h->d_pcg_r, h->d_flags + 1);
  const int max_it = std::max(0, opt.max_linear_solver_iterations);
  launch_pcg_init(s, NC, h->d_pcg_b, h->d_flags + 1, h->d_pcg_state, opt.eta, opt.min_linear_solver_iterations,
                  max_it, h->d_pcg_Minv, h->d_pcg_r, h->d_pcg_z, h->d_pcg_p);
  const int* xptr = h->nxlist > 0 ? h->d_xptr : nullptr;
  // the CG update: spread over work-groups (default) or one work-group (DAB_CG_ONEWG=1)
  const bool onewg = h->knobs.cg_onewg != 0;
  auto update = [&](int mode) {
    if (onewg)
      launch_pcg_update(s, NC, mode, h->d_pcg_Ad, h->d_pcg_w, xptr, h->d_xlist, h->d_cross_cam, h->Ux(),
                        h->d_scale_c, h->d_pcg_b, h->d_pcg_p, h->d_pcg_q, h->d_yc, h->d_pcg_r, h->d_pcg_state,
                        h->d_pcg_Minv, h->d_pcg_z);
    else
      launch_cg_update(s, NC, mode, h->d_pcg_Ad, h->d_pcg_w, xptr, h->d_xlist, h->d_cross_cam, h->Ux(),
                       h->d_scale_c, h->d_pcg_b, h->d_pcg_p, h->d_pcg_q, h->d_yc, h->d_pcg_r, h->d_pcg_state,
                       h->d_pcg_Minv, h->d_pcg_z, h->d_cg_partial, h->d_cg_cnt, h->cg_wpart, h->mf_grid_n);
  };
  // CG iterations are enqueued in batches between reads of the device-side state. The
  // first batch is the previous solve's count + 2 (counts change slowly between LM
  // iterations); a finished CG turns the rest of a batch into no-op launches (~4.5 us
  // each), a read costs a host round trip (~25 us).
  int done = 0, batch = std::min(32, std::max(2, h->pcg_hint + 2));
  for (;;) {
    for (int j = 0; j < batch && done < max_it; ++j) {
      ++done;
      CHECK_RC(pcg_matvec(h, yb, h->d_pcg_p));
      const bool reset = done % 10 == 0;  // r = b - S x every 10th iteration
      update(reset ? 1 : 0);
      if (reset) {
        CHECK_RC(pcg_matvec(h, yb, h->d_yc, true));
        update(2);
      }
    }
    HIP_OK(hipMemcpyAsync(h->h_pcg_state, h->d_pcg_state, sizeof(PcgState), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    if (h->h_pcg_state->status != kPcgRunning || done >= max_it) break;
    batch = batch < 4 ? 4 : std::min(2 * batch, 32);
  }
  h->pcg_hint = h->h_pcg_state->iter;
  *iters = h->h_pcg_state->iter;
  *status = h->h_pcg_state->status;
  return 0;
}

extern "C" int dab_update_parameters(dab_handle* h, const double* points, const double* ext) {
  clear_error();
  if (!h || !h->have_problem) return set_error(DAB_E_STATE, "no problem set");
  HIP_OK(hipSetDevice(h->device));
  if (points) {
    std::vector<double> pts((size_t)3 * h->NP);
    for (int i = 0; i < h->NP; ++i)
      for (int k = 0; k < 3; ++k) pts[3 * (size_t)i + k] = points[3 * (size_t)h->pt_of[i] + k];
    HIP_OK(hipMemcpyAsync(h->d_points, pts.data(), pts.size() * sizeof(double), hipMemcpyHostToDevice, h->stream));
    HIP_OK(hipStreamSynchronize(h->stream));
  }
  if (ext) {
    HIP_OK(hipMemcpyAsync(h->d_ext, ext, sizeof(double) * 6 * (size_t)h->E, hipMemcpyHostToDevice, h->stream));
    HIP_OK(hipStreamSynchronize(h->stream));
  }
  return 0;
}

extern "C" int dab_get_parameters(dab_handle* h, double* points, double* ext) {
  clear_error();
  if (!h || !h->have_problem) return set_error(DAB_E_STATE, "no problem set");
  HIP_OK(hipSetDevice(h->device));
  if (points) {
    std::vector<double> pts((size_t)3 * h->NP);
    HIP_OK(hipMemcpyAsync(pts.data(), h->d_points, pts.size() * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HIP_OK(hipStreamSynchronize(h->stream));
    for (int i = 0; i < h->NP; ++i)
      for (int k = 0; k < 3; ++k) points[3 * (size_t)h->pt_of[i] + k] = pts[3 * (size_t)i + k];
  }
  if (ext) {
    HIP_OK(hipMemcpyAsync(ext, h->d_ext, sizeof(double) * 6 * (size_t)h->E, hipMemcpyDeviceToHost, h->stream));
    HIP_OK(hipStreamSynchronize(h->stream));
  }
  return 0;
}

// ------------------------------------------------------------------------------------
// evaluation building blocks
// ------------------------------------------------------------------------------------
// The evaluation pass proper (the benchmark "step"), matrix-free. The camera side goes
// first (k_eval_cams -> U, g_c; k_eval_cross -> arc∘ring blocks) so that, on several
// GPUs, its RCCL all-reduce runs on comm_stream while the point-side kernel
// (k_eval_points -> V, g, cost) runs on the main stream. Expects the camera tables of
// the current x in d_camtab. ev_mid / ev_end (nullable) bracket the point kernel.
// camtab_ready: the caller has just built the camera tables (the LM step needs them for
// later passes); otherwise they are built here only if a pass of this problem reads them.
static int eval_pass(dab_handle* h, bool camtab_ready, hipEvent_t ev_mid = nullptr, hipEvent_t ev_end = nullptr,
                     hipEvent_t ev_pair0 = nullptr, hipEvent_t ev_pair1 = nullptr, bool* pair_rec = nullptr) {
  hipStream_t s = h->stream;
  const DevView& v = h->view;
  bool overlapped = false;
  if (!h->knobs.eval_side_ok())
    return set_error(DAB_E_INVALID, "DAB_EVAL_SIDE=" + std::to_string(h->knobs.eval_side) +
                                        " is a timing ablation (wrong results): only -DDAB_ABLATIONS builds run it");
  // the fused pass reads the tables when the caller has them (the LM loop) — C3: 21.3
  // against 23.2 us per launch — but does not launch a table build of its own for them
  // (k_cam_tables in front of the pass cost more than it saves: 25.6 against 23.9 us per
  // step), unless DAB_FUSED_TAB=1 asks for it
  const bool fused_tab = h->fused && (h->knobs.fused_tab > 0 || (h->knobs.fused_tab < 0 && camtab_ready));
  const bool need_tab = (h->NC > 0 && (h->chunks.ngen > 0 || h->ncross > 0)) || eval_points_needs_camtab(h->eval_wps) ||
                        fused_tab;
  if (!camtab_ready && need_tab) launch_cam_tables(s, h->E, h->d_ext, h->d_camtab);
  const bool fx = h->fused || eval_points_fx(h->eval_wps);
  if (fx) h->fx_last ^= 1;  // this pass adds into set fx_last and zeroes the other
  h->cost_fx_pending = fx;
  if (h->fused && !h->fused_split && ev_mid) HIP_OK(hipEventRecord(ev_mid, s));
  // k_eval_bal: both traversal orders in one launch (side 0), or one side per launch
  auto eval_fused = [&](int grid, int side) {
    launch_eval_bal(s, v, h->d_chunk_beg, h->d_points, h->d_ext, fused_tab ? h->d_camtab : nullptr, h->d_V, h->d_g,
                    h->ug(), h->cost_fx(h->fx_last), h->cost_fx(h->fx_last ^ 1), h->xerr(), grid, side);
  };
  // DAB_EVAL_SIDE=7: the test's frame wait that never completes; ablation builds: 1..6
  const int test_flag = h->knobs.eval_side == 7 ? kSideTestTimeout : 0;
  if (h->fused && !h->fused_split) {  // both halves of the pass in one launch
    eval_fused(h->ncu, h->knobs.eval_side == 7 ? kSideBoth | test_flag : h->knobs.eval_side);
    if (ev_end) HIP_OK(hipEventRecord(ev_end, s));
    if (h->NC > 0) CHECK_RC(h->allreduce(h->d_camred, h->camred_count(), ncclSum));
    return 0;
  }
  if (h->fused) {
    // several ranks: the same kernel as two launches, the camera side first so that its
    // RCCL all-reduce runs on the communication stream during the point side (which
    // leaves one CU per XCD free for it: eval_grid)
    if (ev_mid) HIP_OK(hipEventRecord(ev_mid, s));
    eval_fused(h->ncu, kSideCams | test_flag);
    bool ovl = false;
    if (h->can_overlap()) {
      HIP_OK(hipEventRecord(h->ev_cam, s));
      HIP_OK(hipStreamWaitEvent(h->comm_stream, h->ev_cam, 0));
      CHECK_RC(h->allreduce_comm_stream(h->d_camred, h->camred_count()));
      HIP_OK(hipEventRecord(h->ev_comm, h->comm_stream));
      ovl = true;
    } else {
      CHECK_RC(h->allreduce(h->d_camred, h->camred_count(), ncclSum));
    }
    eval_fused(h->eval_grid, kSidePoints);
    if (ev_end) HIP_OK(hipEventRecord(ev_end, s));
    if (ovl) HIP_OK(hipStreamWaitEvent(s, h->ev_comm, 0));
    return 0;
  }
  if (h->NC > 0 && h->pair_eval) {
    // the composed observations pair-major (camera halves + cross blocks in one pass),
    // the other entries camera-major, then one fixed-order sum per camera
    DevView v2 = v;
    v2.cm_idx = h->d_cm2_idx;
    v2.cm_xy = h->d_cm2_xy;
    launch_eval_cams_gen(s, v2, h->nchunk2, h->d_chunk2_beg, h->d_points, h->d_ext, h->d_camtab, h->d_partial2);
    if (ev_pair0) HIP_OK(hipEventRecord(ev_pair0, s));
    launch_eval_pair(s, v, h->nxchunk, h->d_xchunk_beg, h->d_x_idx, h->d_x_xy, h->d_points, h->d_camtab,
                     h->d_xpartial, h->d_xcpart, h->pair_uni_intr);
    if (ev_pair1) HIP_OK(hipEventRecord(ev_pair1, s));
    if (pair_rec) *pair_rec = ev_pair0 && ev_pair1 && h->nxchunk > 0;
    launch_cam_final(s, h->NC, h->d_seg2_chunk, h->d_partial2, h->d_xcam_ptr, h->d_xcam_list, h->d_xcpart, h->ug());
    launch_seg_final(s, h->ncross, 36, h->d_xseg_chunk, h->d_xpartial, h->Ux(), h->max_xseg_chunks);
  } else if (h->NC > 0) {
    // one chunk per camera: the chunk kernels write the camera rows directly
    const bool direct = h->nchunk == h->NC;
    launch_eval_cams(s, v, h->chunks, h->d_chunk_beg, h->d_points, h->d_ext, h->d_camtab,
                     direct ? h->ug() : h->d_partial);
    if (!direct) launch_seg_final(s, h->NC, 27, h->d_seg_chunk, h->d_partial, h->ug(), h->max_seg_chunks);
  }
  if (h->NC > 0) {
    if (h->ncross > 0 && !h->pair_eval) {
      if (h->nxchunk > 0) {
        launch_eval_cross(s, v, h->nxchunk, h->d_xchunk_beg, h->d_x_idx, h->d_x_xy, h->d_points, h->d_camtab,
                          h->d_xpartial);
        launch_seg_final(s, h->ncross, 36, h->d_xseg_chunk, h->d_xpartial, h->Ux(), h->max_xseg_chunks);
      } else {
        HIP_OK(hipMemsetAsync(h->Ux(), 0, sizeof(double) * 36 * (size_t)h->ncross, s));
      }
    }
    if (h->can_overlap()) {
      HIP_OK(hipEventRecord(h->ev_cam, s));
      HIP_OK(hipStreamWaitEvent(h->comm_stream, h->ev_cam, 0));
      CHECK_RC(h->allreduce_comm_stream(h->d_camred, h->camred_count()));
      HIP_OK(hipEventRecord(h->ev_comm, h->comm_stream));
      overlapped = true;
    } else {
      CHECK_RC(h->allreduce(h->d_camred, h->camred_count(), ncclSum));
    }
  }
  if (ev_mid) HIP_OK(hipEventRecord(ev_mid, s));
  launch_eval_points(s, h->view, h->d_points, h->d_ext, h->d_camtab, h->d_V, h->d_g, h->d_gpart, h->d_arrivals,
                     h->d_scal + S_COST, h->cost_fx(h->fx_last), h->cost_fx(h->fx_last ^ 1), h->eval_grid,
                     h->eval_wps);
  if (ev_end) HIP_OK(hipEventRecord(ev_end, s));
  if (overlapped) HIP_OK(hipStreamWaitEvent(s, h->ev_comm, 0));
  return 0;
}

// Residual + Jacobian at the current x and the J^T J / J^T r blocks (camera side
// all-reduced). Leaves cost / gradient scalars in d_scal (point parts all-reduced).
// tables_current: d_camtab already holds the tables of d_ext (after an accepted step, the
// candidate's tables swapped in with its parameters), so none are built here
static int eval_jacobian_and_blocks(dab_handle* h, bool with_norms, bool tables_current = false) {
  hipStream_t s = h->stream;
  if (!tables_current) launch_cam_tables(s, h->E, h->d_ext, h->d_camtab);
  CHECK_RC(eval_pass(h, true));
  if (with_norms) {
    launch_grad_points(s, h->NP, h->d_points, h->d_g, h->d_gpart, h->red_grid);
    launch_final_sum(s, h->red_grid, 3, h->d_gpart, h->d_scal + S_GMAX_P, 1u);
    launch_cam_norms(s, h->E, h->d_ext_col, h->d_ext, nullptr, h->NC > 0 ? h->ug() : nullptr,
                     h->d_scal + S_CAM0);
  }
  // cross-rank: sums of cost, bad, gnorm, xnorm; max of gmax
  CHECK_RC(h->allreduce_cost());
  if (with_norms) {
    CHECK_RC(h->allreduce(h->d_scal + S_GMAX_P, 1, ncclMax));
    CHECK_RC(h->allreduce(h->d_scal + S_GNORM_P, 2, ncclSum));
  }
  return 0;
}

// k_eval_bal's error bits: a bounded work-group wait timed out, the pass's results are void
static int xerr_fail(unsigned long long e) {
  return set_error(DAB_E_DEVICE, "evaluation pass: a work-group wait timed out (code " + std::to_string(e) + ")");
}
// the handle's sticky error word (dab_sync after bench passes), cleared once read
static int xerr_check_sticky(dab_handle* h) {
  unsigned e = 0;
  std::memcpy(&e, h->h_scal + S_XERR, sizeof(e));
  if (e == 0) return 0;
  HIP_OK(hipMemsetAsync(h->d_scal + S_XERR, 0, sizeof(double), h->stream));
  HIP_OK(hipStreamSynchronize(h->stream));
  return xerr_fail(e);
}
static int read_scalars(dab_handle* h) {
  HIP_OK(hipMemcpyAsync(h->h_scal, h->d_scal, sizeof(double) * S_NSLOTS, hipMemcpyDeviceToHost, h->stream));
  HIP_OK(hipMemcpyAsync(h->h_flags, h->d_flags, sizeof(int) * 4, hipMemcpyDeviceToHost, h->stream));
  HIP_OK(hipStreamSynchronize(h->stream));
  // a one-shot all-reduce that gave up waiting for a peer poisons its output: stop here,
  // before any decision is taken on it (every rank's next call fails the same way)
  CHECK_RC(p2p_check(h->p2p_main));
  CHECK_RC(p2p_check(h->p2p_comm));
  if (h->cost_fx_pending) {
    // the last evaluation pass left its cost in fixed point (cost_fx_commit): exact
    // integer limb sums, converted once here. Its error bits (kFxErr) were summed over the
    // ranks with the cost (allreduce_cost), so a wait that ran out on any rank fails this
    // call on every rank, before any decision is taken on the pass
    unsigned long long w[kFxWords];
    std::memcpy(w, h->h_scal + S_CFX + (size_t)kFxWords * h->fx_last, sizeof(w));
    h->cost_fx_pending = false;
    if (const unsigned long long e = cost_fx_err(w)) {
      HIP_OK(hipMemsetAsync(h->d_scal + S_XERR, 0, sizeof(double), h->stream));  // reported here
      HIP_OK(hipStreamSynchronize(h->stream));
      return xerr_fail(e);
    }
    cost_fx_total(w, h->h_scal[S_COST], h->h_scal[S_COST_BAD]);
  }
  return 0;
}

// Jacobi scaling s = 1/(1+sqrt(diag(J^T J))), computed once at iteration 0.
__global__ void k_scale_points(int NP, const double* __restrict__ V, double* __restrict__ sp, int on) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 3 * NP) return;
  const int k = i / NP, p = i - k * NP;
  const int vi = k == 0 ? 0 : (k == 1 ? 3 : 5);
  sp[i] = on ? 1.0 / (1.0 + sqrt(V[(size_t)vi * NP + p])) : 1.0;
}
__global__ void k_scale_cams(int NC, const double* __restrict__ ug, double* __restrict__ sc, int on) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 6 * NC) return;
  const int c = i / 6, a = i - 6 * c;
  const int q = a * 6 - (a * (a - 1)) / 2;  // (a,a) in the packed upper layout
  sc[i] = on ? 1.0 / (1.0 + sqrt(ug[27 * (size_t)c + q])) : 1.0;
}

static void print_header() {
  std::printf("iter      cost      cost_change  |gradient|   |step|    tr_ratio  tr_radius  ls_iter  iter_time  total_time\n");
}
static void print_iter(const dab_iteration& it, double total) {
  std::printf("%4d % 3.6e % 3.2e % 3.2e % 3.2e % 3.2e % 3.2e %4d % 3.2e % 3.2e\n", it.iteration, it.cost,
              it.cost_change, it.gradient_max_norm, it.step_norm, it.relative_decrease, it.trust_region_radius,
              it.linear_solver_iterations, it.iteration_time_in_seconds, total);
  std::fflush(stdout);
}

// Wall-clock since solve start, maxed over ranks so every rank takes the
// "Maximum solver time reached" exit on the same iteration. Returns < 0 on error.
static double elapsed_collective(dab_handle* h, double local) {
  if (!h->coll()) return local;
  hipStream_t s = h->stream;
  h->h_scal[S_TIME] = local;
  if (hipMemcpyAsync(h->d_scal + S_TIME, &h->h_scal[S_TIME], sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess)
    return -1.0;
  if (h->allreduce(h->d_scal + S_TIME, 1, ncclMax) != 0) return -1.0;
  if (hipMemcpyAsync(&h->h_scal[S_TIME], h->d_scal + S_TIME, sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess)
    return -1.0;
  if (hipStreamSynchronize(s) != hipSuccess) return -1.0;
  return h->h_scal[S_TIME];
}

// ------------------------------------------------------------------------------------
// dab_solve: the trust-region LM loop
// ------------------------------------------------------------------------------------
static int solve_impl(dab_handle* h, const dab_options* opt_in, dab_summary* sum);
extern "C" int dab_solve(dab_handle* h, const dab_options* opt_in, dab_summary* sum) {
  const int rc = solve_impl(h, opt_in, sum);
  CHECK_RC(guard_fail(h, "dab_solve"));
  return rc;
}
static int solve_impl(dab_handle* h, const dab_options* opt_in, dab_summary* sum) {
  clear_error();
  if (!h || !h->have_problem) return set_error(DAB_E_STATE, "no problem set");
  if (!sum) return set_error(DAB_E_INVALID, "null summary");
  dab_options opt;
  if (opt_in) opt = *opt_in;
  else dab_options_init(&opt);
  if (opt.linear_solver_type != DAB_LINEAR_SOLVER_EXPLICIT_SCHUR &&
      opt.linear_solver_type != DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG &&
      opt.linear_solver_type != DAB_LINEAR_SOLVER_AUTO)
    return set_error(DAB_E_INVALID, "unknown linear_solver_type");
  if (opt.linear_solver_type == DAB_LINEAR_SOLVER_AUTO)  // the same choice on every rank (NC is the union's)
    opt.linear_solver_type = h->world <= 1 || h->NC == 0 || mf_schur_fits(h->NC, h->E, h->NI)
                                 ? DAB_LINEAR_SOLVER_EXPLICIT_SCHUR
                                 : DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG;
  const bool use_pcg = opt.linear_solver_type == DAB_LINEAR_SOLVER_IMPLICIT_SCHUR_PCG;
  HIP_OK(hipSetDevice(h->device));
  static const bool timing = getenv("DAB_SETUP_TIMING") != nullptr;
  const double tp0 = now_s();
  CHECK_RC(use_pcg ? build_pcg_buffers(h) : build_schur_tables(h));
  const double tp1 = now_s();
  // the dense factorisation's scratch and captured graph belong to the set-up, not to the
  // first LM iteration (kept while the camera count and the buffers stay the same)
  if (!use_pcg && h->NC > 0 &&
      chol_prepare(h->chol, h->stream, 6 * h->NC, h->d_S, h->lds, h->d_yc, h->d_flags + 1) != 0)
    return set_error(DAB_E_DEVICE, "dense Cholesky set-up failed");
  if (timing)
    std::fprintf(stderr, "solve prep: %s %.2f ms, Cholesky graph %.2f ms\n", use_pcg ? "pcg buffers" : "schur tables",
                 1e3 * (tp1 - tp0), 1e3 * (now_s() - tp1));
  // Y records of each step: fp64 (both layouts), or fp32 for the mixed-precision PCG
  // (Jacobians, residuals, V/U/g, the CG vectors and scalars stay fp64)
  // (the matrix-free PCG of small camera sets stores no Y and is all fp64)
  const bool y32 = use_pcg && opt.pcg_fp32 != 0 && !h->mf;
  // matrix-free mixed precision: fp32 products, fp64 sums, recurrences and true residuals
  h->mf32 = use_pcg && opt.pcg_fp32 != 0 && h->mf;
  if (y32 && !h->d_Y32c) {
    CHECK_RC(h->dev.alloc(&h->d_Y32c, (size_t)kYRec * std::max(1, h->NE)));
    CHECK_RC(h->dev.alloc(&h->d_Y32p, (size_t)kYRec * std::max(1, h->NS) * (h->any_compose ? 2 : 1)));
  }
  const YBufs yb = y32 ? YBufs{h->d_Y32c, h->d_Y32p, true} : YBufs{h->d_Y, h->d_Yp, false};
  hipStream_t s = h->stream;
  const DevView& v = h->view;
  const int NP = h->NP, NC = h->NC, n = 6 * NC;
  const double t_start = now_s();
  std::memset(sum->message, 0, sizeof(sum->message));
  sum->iterations_written = 0;
  sum->num_successful_steps = sum->num_unsuccessful_steps = 0;
  sum->num_iterations = 0;
  sum->num_residuals = 2 * h->N;
  sum->num_parameters = 3 * NP + 6 * NC;
  sum->num_free_points = NP;
  sum->num_free_ext = NC;
  sum->jacobian_evaluation_time_in_seconds = 0;
  sum->residual_evaluation_time_in_seconds = 0;
  sum->linear_solver_time_in_seconds = 0;
  sum->termination_type = DAB_FAILURE;
  sum->linear_solver_type_used = opt.linear_solver_type;
  sum->schur_assembly = use_pcg ? (h->mf ? (h->mf32 ? DAB_PCG_MATRIX_FREE_FP32 : DAB_PCG_MATRIX_FREE) : DAB_PCG_STORED_Y)
                                : (h->schur_tiles ? DAB_SCHUR_TILES : DAB_SCHUR_PAIRS);
  const bool verbose = opt.minimizer_progress_to_stdout && h->rank == 0;
  const bool in_global = true;  (void)in_global;

  // ---- iteration 0 ----
  // a solve starts with a clean sticky error word (a timed-out wait of an earlier call was
  // reported by that call)
  HIP_OK(hipMemsetAsync(h->d_scal + S_XERR, 0, sizeof(double), s));
  double t0 = now_s();
  CHECK_RC(eval_jacobian_and_blocks(h, true));
  CHECK_RC(read_scalars(h));
  if (timing) std::fprintf(stderr, "solve iteration 0: %.2f ms\n", 1e3 * (now_s() - t0));
  {
    const int g3 = grid_for(3 * NP, 256, 1 << 20);
    k_scale_points<<<g3, 256, 0, s>>>(NP, h->d_V, h->d_scale_p, opt.jacobi_scaling);
    if (NC > 0) k_scale_cams<<<grid_for(6 * NC, 256, 1 << 20), 256, 0, s>>>(NC, h->ug(), h->d_scale_c, opt.jacobi_scaling);
  }
  sum->jacobian_evaluation_time_in_seconds += now_s() - t0;
  double x_cost = 0.5 * h->h_scal[S_COST];
  bool eval_ok = h->h_scal[S_COST_BAD] == 0.0;
  double gmax = std::max(h->h_scal[S_GMAX_P], h->h_scal[S_CAM0 + 2]);
  double x_norm = std::sqrt(h->h_scal[S_XNORM_P] + h->h_scal[S_CAM0 + 4]);
  sum->initial_cost = x_cost;
  double final_cost = x_cost;
  if (!eval_ok) {
    std::snprintf(sum->message, sizeof(sum->message), "Residual and Jacobian evaluation failed.");
    sum->final_cost = x_cost;
    sum->total_time_in_seconds = now_s() - t_start;
    return 0;
  }

  // best state (Ceres keeps parameters_ = the lowest-cost accepted x)
  double minimum_cost = x_cost;
  int iteration = 0;
  double radius = opt.initial_trust_region_radius, decrease_factor = 2.0;
  int num_invalid = 0;
  int term = -1;
  dab_iteration it{};
  it.iteration = 0;
  it.step_is_successful = 1;
  it.step_is_valid = 1;
  it.cost = x_cost;
  it.gradient_max_norm = gmax;
  double iter_start = t_start;
  if (verbose) print_header();

  for (;;) {
    // FinalizeIterationAndCheckIfMinimizerCanContinue
    if (it.step_is_successful) {
      sum->num_successful_steps++;
      if (x_cost < minimum_cost) minimum_cost = x_cost;
    } else {
      sum->num_unsuccessful_steps++;
    }
    it.trust_region_radius = radius;
    it.iteration_time_in_seconds = now_s() - iter_start;
    if (it.cost < final_cost) final_cost = it.cost;
    if (sum->iterations && sum->iterations_written < sum->iterations_capacity)
      sum->iterations[sum->iterations_written++] = it;
    if (verbose) print_iter(it, now_s() - t_start);
    sum->num_iterations = iteration;
    const double elapsed = elapsed_collective(h, now_s() - t_start);
    if (elapsed < 0) return set_error(DAB_E_DEVICE, "solver-time all-reduce failed");
    if (elapsed >= opt.max_solver_time_in_seconds) {
      term = DAB_NO_CONVERGENCE;
      std::snprintf(sum->message, sizeof(sum->message), "Maximum solver time reached.");
      break;
    }
    if (iteration >= opt.max_num_iterations) {
      term = DAB_NO_CONVERGENCE;
      std::snprintf(sum->message, sizeof(sum->message),
                    "Maximum number of iterations reached. Number of iterations: %d.", iteration);
      break;
    }
    if (it.step_is_successful && gmax <= opt.gradient_tolerance) {
      term = DAB_CONVERGENCE;
      std::snprintf(sum->message, sizeof(sum->message), "Gradient tolerance reached. Gradient max norm: %e <= %e",
                    gmax, opt.gradient_tolerance);
      break;
    }
    if (radius <= opt.min_trust_region_radius) {
      term = DAB_CONVERGENCE;
      std::snprintf(sum->message, sizeof(sum->message), "Minimum trust region radius reached.");
      break;
    }

    iter_start = now_s();
    iteration++;
    const double prev_gmax = gmax;
    it = dab_iteration{};
    it.iteration = iteration;
    it.linear_solver_iterations = 1;

    // ---- ComputeTrustRegionStep (DENSE_SCHUR) ----
    const double tls = now_s();
    StepScalars sc{radius, opt.min_lm_diagonal, opt.max_lm_diagonal};
    HIP_OK(hipMemsetAsync(h->d_flags, 0, sizeof(int) * 4, s));
    launch_point_factor(s, v, h->d_V, h->d_g, h->d_scale_p, sc, h->d_L, h->d_q, h->d_flags);
    bool pcg_fail = false;
    if (NC > 0 && use_pcg) {
      if (!h->mf) launch_entry_y(s, v, h->d_points, h->d_camtab, h->d_scale_c, h->d_L, yb, true);
      int cg_iters = 0, cg_status = 0;
      CHECK_RC(pcg_solve(h, opt, sc, yb, &cg_iters, &cg_status));
      it.linear_solver_iterations = cg_iters;
      pcg_fail = cg_status == kPcgFailure;
    } else if (NC > 0 && h->schur_tiles) {
      // S by register-owned block tiles over the records' Y (re-evaluated once per step)
      SchurTiles a = h->tiles;
      a.kq = 0;
      if (x_cost > 0.0 && std::isfinite(x_cost)) {
        int e2;
        (void)std::frexp(2.0 * x_cost, &e2);  // sum_p |q_p|^2 <= 2 cost < 2^e2
        a.kq = (e2 + 1) >> 1;
      }
      launch_schur_scale(s, NC, h->ug(), h->d_scale_c, h->d_kx);
      HIP_OK(hipMemsetAsync(h->d_rfx, 0, sizeof(unsigned long long) * 6 * (size_t)NC, s));
      launch_schur_y(s, v, h->d_points, h->d_camtab, h->d_L, h->d_q, h->d_scale_c, a, h->d_yrec, h->d_rfx);
      launch_schur_tiles(s, h->d_yrec, a, NC);
      launch_schur_sum_tiles(s, a, h->d_sblk);
      CHECK_RC(h->allreduce(h->d_sblk, (size_t)a.nelem, ncclSum));
      CHECK_RC(h->allreduce_u64(reinterpret_cast<uint64_t*>(h->d_rfx), (size_t)6 * NC));
      HIP_OK(hipMemsetAsync(h->d_S, 0, sizeof(double) * (size_t)(n + 1) * h->lds, s));
      launch_schur_unpack(s, NC, h->d_sblk, h->d_rfx, h->d_kx, a.kq, h->d_S, h->lds, h->ybc());
      launch_s_add_u(s, NC, h->ug(), h->ncross, h->d_cross_cam, h->Ux(), h->d_scale_c, sc, h->ybc(), h->d_S, h->lds);
      if (chol_factor_solve(h->chol, s, n, h->d_S, h->lds, h->d_yc, h->d_flags + 1) != 0)
        return set_error(DAB_E_DEVICE, "dense Cholesky launch failed");
    } else if (NC > 0) {
      // fp64 Y: the camera-major pass writes the [NE][18] records the S blocks gather (no
      // plane-to-record copy); the slot planes as before (back substitution)
      const bool rec = !yb.f32;
      launch_entry_y(s, v, h->d_points, h->d_camtab, h->d_scale_c, h->d_L, yb, true, rec ? h->d_Yrec : nullptr);
      // one rank: the S blocks straight into the dense S (nothing to all-reduce), no zero
      // fill of the whole matrix and no scatter; several: packed, all-reduced, unpacked
      const bool direct = h->world == 1;
      launch_s_blocks(s, h->nblk, h->d_blk_pair_beg, h->d_pairs, rec ? nullptr : h->d_Y, h->NE, h->packed(),
                      h->d_Yrec, direct ? h->d_S : nullptr, h->lds, h->d_blk_cam, h->nzero, h->d_blk_zero);
      launch_cam_rhs_partial(s, v, h->nchunk, h->d_chunk_beg, rec ? h->d_Yrec : h->d_Y, h->d_q, h->d_partial, rec);
      launch_seg_final(s, NC, 6, h->d_seg_chunk, h->d_partial, h->ybc(), h->max_seg_chunks);
      if (direct) {
        launch_s_add_u(s, NC, h->ug(), h->ncross, h->d_cross_cam, h->Ux(), h->d_scale_c, sc, h->ybc(), h->d_S,
                       h->lds);
      } else {
        CHECK_RC(h->allreduce(h->d_spack, h->spack_count(), ncclSum));
        launch_s_unpack(s, NC, h->nblk, h->d_blk_cam, h->packed(), h->ug(), h->ncross, h->d_cross_cam, h->Ux(),
                        h->d_scale_c, sc, h->ybc(), h->d_S, h->lds);
      }
      if (chol_factor_solve(h->chol, s, n, h->d_S, h->lds, h->d_yc, h->d_flags + 1) != 0)
        return set_error(DAB_E_DEVICE, "dense Cholesky launch failed");
    }
    if ((use_pcg && h->mf) || (!use_pcg && h->schur_tiles))
      launch_mf_backsub(s, v, h->d_points, h->d_camtab, h->d_scale_c, h->d_L, h->d_q, h->d_yc, h->d_dp, h->mf_grid_n);
    else
      launch_backsub(s, v, h->d_L, h->d_q, yb, NC > 0 ? h->d_yc : nullptr, h->d_dp);
    // candidate x + delta and the model / candidate cost in one observation pass
    launch_axpy_points(s, NP, h->d_points, h->d_dp, h->d_points_c, h->d_gpart, h->red_grid);
    launch_final_sum(s, h->red_grid, 2, h->d_gpart, h->d_scal + S_STEP_P);
    launch_cam_candidate(s, h->E, h->d_ext_col, h->d_ext, NC > 0 ? h->d_yc : nullptr, h->d_scale_c, h->d_ext_c,
                         h->d_dc);
    launch_cam_norms(s, h->E, h->d_ext_col, h->d_ext, h->d_ext_c, nullptr, h->d_scal + S_CAM0);
    launch_cam_tables(s, h->E, h->d_ext_c, h->d_camtab_c);
    const double tre = now_s();
    launch_candidate(s, v, h->d_points, h->d_camtab, h->d_dp, h->d_dc, h->d_camtab_c, h->d_gpart, h->red_grid);
    launch_final_sum(s, h->red_grid, 3, h->d_gpart, h->d_scal + S_MODEL);
    CHECK_RC(h->allreduce(h->d_scal + S_MODEL, 5, ncclSum));
    CHECK_RC(h->allreduce_max_i32(h->d_flags, 4));
    CHECK_RC(read_scalars(h));
    // bit 2 of the Cholesky flag: a bounded wait inside the factorisation gave up (a
    // scheduling / residency fault, not a property of the matrix): an error, not a
    // rejected step (bit 1 = not positive definite)
    if (!use_pcg && NC > 0 && (h->h_flags[1] & 2))
      return set_error(DAB_E_DEVICE, "dense Cholesky: a bounded wait between work-groups timed out");
    const double tdone = now_s();
    sum->linear_solver_time_in_seconds += tre - tls;
    sum->residual_evaluation_time_in_seconds += tdone - tre;

    const bool solve_fail = pcg_fail || h->h_flags[0] != 0 || h->h_flags[1] != 0 || h->h_flags[2] != 0 ||
                            h->h_flags[3] != 0;
    const double model_cost_change = h->h_scal[S_MODEL];
    it.step_is_valid = !solve_fail && std::isfinite(model_cost_change) && model_cost_change > 0.0;
    if (!it.step_is_valid) {
      num_invalid++;
      if (num_invalid >= opt.max_num_consecutive_invalid_steps) {
        term = DAB_FAILURE;
        std::snprintf(sum->message, sizeof(sum->message),
                      "Number of consecutive invalid steps more than Solver::Options::max_num_consecutive_invalid_steps: %d",
                      opt.max_num_consecutive_invalid_steps);
        break;
      }
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
      it.cost = x_cost;
      it.gradient_max_norm = prev_gmax;
      it.step_is_successful = 0;
      continue;
    }
    num_invalid = 0;
    const double candidate_cost = h->h_scal[S_CAND_BAD] != 0.0 ? 1.7976931348623157e308 : 0.5 * h->h_scal[S_CAND];
    // ParameterToleranceReached
    it.step_norm = std::sqrt(h->h_scal[S_STEP_P] + h->h_scal[S_CAM0 + 0]);
    if (it.step_norm <= opt.parameter_tolerance * (x_norm + opt.parameter_tolerance)) {
      term = DAB_CONVERGENCE;
      std::snprintf(sum->message, sizeof(sum->message), "Parameter tolerance reached. Relative step_norm: %e <= %e.",
                    it.step_norm / (x_norm + opt.parameter_tolerance), opt.parameter_tolerance);
      break;
    }
    // FunctionToleranceReached
    it.cost_change = x_cost - candidate_cost;
    if (std::fabs(it.cost_change) <= opt.function_tolerance * x_cost) {
      term = DAB_CONVERGENCE;
      std::snprintf(sum->message, sizeof(sum->message), "Function tolerance reached. |cost_change|/cost: %e <= %e",
                    std::fabs(it.cost_change) / x_cost, opt.function_tolerance);
      break;
    }
    it.relative_decrease = (x_cost - candidate_cost) / model_cost_change;
    if (it.relative_decrease > opt.min_relative_decrease) {
      // HandleSuccessfulStep: x <- candidate, re-evaluate J at the new point
      const double xc_norm = std::sqrt(h->h_scal[S_XCNORM_P] + h->h_scal[S_CAM0 + 1]);
      std::swap(h->d_points, h->d_points_c);
      std::swap(h->d_ext, h->d_ext_c);
      std::swap(h->d_camtab, h->d_camtab_c);  // the candidate pass built the tables of x + delta
      x_norm = xc_norm;
      const double tj = now_s();
      CHECK_RC(eval_jacobian_and_blocks(h, true, true));
      CHECK_RC(read_scalars(h));
      sum->jacobian_evaluation_time_in_seconds += now_s() - tj;
      if (h->h_scal[S_COST_BAD] != 0.0) {
        term = DAB_FAILURE;
        std::snprintf(sum->message, sizeof(sum->message), "Residual and Jacobian evaluation failed.");
        break;
      }
      x_cost = 0.5 * h->h_scal[S_COST];
      gmax = std::max(h->h_scal[S_GMAX_P], h->h_scal[S_CAM0 + 2]);
      it.step_is_successful = 1;
      it.cost = x_cost;
      it.gradient_max_norm = gmax;
      radius = radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * it.relative_decrease - 1.0, 3));
      radius = std::min(opt.max_trust_region_radius, radius);
      decrease_factor = 2.0;
    } else {
      it.step_is_successful = 0;
      it.cost = candidate_cost;
      it.gradient_max_norm = prev_gmax;
      radius = radius / decrease_factor;
      decrease_factor *= 2.0;
    }
  }

  sum->termination_type = term;
  sum->final_cost = final_cost;
  (void)minimum_cost;
  // the accepted iterate is always the lowest-cost one (steps are monotone), so the
  // device-resident x is Ceres' parameters_; write it back (sfm.cc:47-48 semantics)
  HIP_OK(hipStreamSynchronize(s));
  CHECK_RC(p2p_check(h->p2p_main));  // fail closed: the caller's arrays stay untouched
  CHECK_RC(p2p_check(h->p2p_comm));
  CHECK_RC(dab_get_parameters(h, h->prob.points, h->prob.ext));
  sum->total_time_in_seconds = now_s() - t_start;
  return 0;
}

// ------------------------------------------------------------------------------------
// evaluation entry points (filterPoint3d residual pass, parity)
// ------------------------------------------------------------------------------------
extern "C" int dab_eval_residuals(dab_handle* h, double* residuals, double* cost) {
  clear_error();
  if (!h || !h->have_problem) return set_error(DAB_E_STATE, "no problem set");
  HIP_OK(hipSetDevice(h->device));
  hipStream_t s = h->stream;
  launch_cam_tables(s, h->E, h->d_ext, h->d_camtab);
  launch_residual(s, h->view, h->d_points, h->d_camtab, h->d_r, h->d_gpart, h->red_grid);
  launch_final_sum(s, h->red_grid, 2, h->d_gpart, h->d_scal + S_COST);
  h->cost_fx_pending = false;
  CHECK_RC(read_scalars(h));
  if (cost) *cost = 0.5 * h->h_scal[S_COST];
  if (residuals) {
    std::vector<double> r((size_t)2 * h->NS);
    HIP_OK(hipMemcpyAsync(r.data(), h->d_r, r.size() * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    for (int s2 = 0; s2 < h->NS; ++s2) {
      const int o = h->perm[s2];
      if (o < 0) continue;
      residuals[2 * (size_t)o] = r[2 * (size_t)s2];
      residuals[2 * (size_t)o + 1] = r[2 * (size_t)s2 + 1];
    }
  }
  return 0;
}

extern "C" int dab_eval_jacobians(dab_handle* h, double* residuals, double* jacobians) {
  clear_error();
  if (!h || !h->have_problem) return set_error(DAB_E_STATE, "no problem set");
  HIP_OK(hipSetDevice(h->device));
  hipStream_t s = h->stream;
  if (!h->d_Jfull) CHECK_RC(h->dev.alloc(&h->d_Jfull, (size_t)30 * h->NS));
  launch_cam_tables(s, h->E, h->d_ext, h->d_camtab);
  launch_jacobian_full(s, h->view, h->d_points, h->d_camtab, h->d_r, h->d_Jfull);
  std::vector<double> r((size_t)2 * h->NS), J((size_t)30 * h->NS);
  HIP_OK(hipMemcpyAsync(r.data(), h->d_r, r.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(J.data(), h->d_Jfull, J.size() * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  for (int s2 = 0; s2 < h->NS; ++s2) {
    const int o = h->perm[s2];
    if (o < 0) continue;
    if (residuals) {
      residuals[2 * (size_t)o] = r[2 * (size_t)s2];
      residuals[2 * (size_t)o + 1] = r[2 * (size_t)s2 + 1];
    }
    if (jacobians) {
      double* out = jacobians + (size_t)o * 30;
      const bool comp = h->prob.obs_ext1[o] >= 0;
      for (int col = 0; col < 15; ++col)
        for (int row = 0; row < 2; ++row) {
          double val = 0.0;
          if (col < 9 || comp) val = J[(size_t)(2 * col + row) * h->NS + s2];
          out[row * 15 + col] = val;
        }
    }
  }
  return 0;
}

extern "C" int dab_filter(dab_handle* h, double error_boundary, const double center[3], double radius,
                          uint8_t* obs_keep, uint8_t* point_keep, int32_t* n_obs_kept, int32_t* n_points_kept) {
  clear_error();
  if (!h || !h->have_problem) return set_error(DAB_E_STATE, "no problem set");
  if (!center) return set_error(DAB_E_INVALID, "null hemisphere center");
  HIP_OK(hipSetDevice(h->device));
  hipStream_t s = h->stream;
  Dev tmp{"entry-point temporaries"};
  unsigned char *d_slot = nullptr, *d_pt = nullptr;
  CHECK_RC(tmp.alloc(&d_slot, (size_t)std::max(1, h->NS)));
  CHECK_RC(tmp.alloc(&d_pt, (size_t)std::max(1, h->NP)));
  launch_cam_tables(s, h->E, h->d_ext, h->d_camtab);
  launch_filter(s, h->view, h->d_points, h->d_camtab, error_boundary, center, radius, d_slot, d_pt);
  std::vector<unsigned char> slot((size_t)h->NS), pt((size_t)h->NP);
  if (h->NS > 0) HIP_OK(hipMemcpyAsync(slot.data(), d_slot, slot.size(), hipMemcpyDeviceToHost, s));
  if (h->NP > 0) HIP_OK(hipMemcpyAsync(pt.data(), d_pt, pt.size(), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  CHECK_RC(guard_fail(h, "dab_filter", &tmp));
  int32_t no = 0, np = 0;
  if (obs_keep) std::memset(obs_keep, 0, (size_t)h->N);
  for (int s2 = 0; s2 < h->NS; ++s2) {
    const int o = h->perm[s2];
    if (o < 0) continue;
    if (obs_keep) obs_keep[o] = slot[s2];
    no += slot[s2];
  }
  if (point_keep) std::memset(point_keep, 0, (size_t)h->prob.num_points);
  for (int i = 0; i < h->NP; ++i) {
    if (point_keep) point_keep[h->pt_of[i]] = pt[i];
    np += pt[i];
  }
  if (n_obs_kept) *n_obs_kept = no;
  if (n_points_kept) *n_points_kept = np;
  return 0;
}

extern "C" int dab_dense_spd_solve(dab_handle* h, int n, const double* A, const double* b, double* x,
                                   double* factor_ms) {
  clear_error();
  if (!h) return set_error(DAB_E_INVALID, "null handle");
  if (n < 0 || (n > 0 && (!A || !b || !x))) return set_error(DAB_E_INVALID, "bad dense solve arguments");
  if (n == 0) return 0;
  HIP_OK(hipSetDevice(h->device));
  hipStream_t s = h->stream;
  int lds = ((n + 1 + 7) / 8) * 8;
  if (lds % 512 == 0) lds += 8;
  Dev tmp{"entry-point temporaries"};
  double *dA = nullptr, *dy = nullptr;
  int* dflag = nullptr;
  CHECK_RC(tmp.alloc(&dA, (size_t)(n + 1) * lds));
  CHECK_RC(tmp.alloc(&dy, (size_t)n));
  CHECK_RC(tmp.alloc(&dflag, 1));
  HIP_OK(hipMemsetAsync(dA, 0, sizeof(double) * (size_t)(n + 1) * lds, s));
  HIP_OK(hipMemsetAsync(dflag, 0, sizeof(int), s));
  HIP_OK(hipMemcpy2DAsync(dA, lds * sizeof(double), A, n * sizeof(double), n * sizeof(double), n,
                          hipMemcpyHostToDevice, s));
  HIP_OK(hipMemcpyAsync(dA + (size_t)n * lds, b, n * sizeof(double), hipMemcpyHostToDevice, s));
  HIP_OK(hipEventRecord(h->ev0, s));
  if (chol_factor_solve(h->chol, s, n, dA, lds, dy, dflag) != 0)
    return set_error(DAB_E_DEVICE, "dense factorisation launch failed");
  HIP_OK(hipEventRecord(h->ev1, s));
  int flag = 0;
  HIP_OK(hipMemcpyAsync(x, dy, n * sizeof(double), hipMemcpyDeviceToHost, s));
  HIP_OK(hipMemcpyAsync(&flag, dflag, sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  CHECK_RC(guard_fail(h, "dab_dense_spd_solve", &tmp));
  float ms = 0.f;
  HIP_OK(hipEventElapsedTime(&ms, h->ev0, h->ev1));
  if (factor_ms) *factor_ms = ms;
  return flag ? 1 : 0;
}

// ------------------------------------------------------------------------------------
// benchmark hooks
// ------------------------------------------------------------------------------------
// accumulate the timings of the recorded bench steps (waits for the last one)
static int collect_bench_events(dab_handle* h) {
  if (h->bench_pending == 0) return 0;
  HIP_OK(hipEventSynchronize(h->bench_ev[h->bench_pending - 1][3]));
  for (int i = 0; i < h->bench_pending; ++i) {
    const auto& ev = h->bench_ev[i];
    float a = 0.f, b = 0.f, c = 0.f;
    HIP_OK(hipEventElapsedTime(&a, ev[0], ev[1]));  // camera side (+ all-reduce issue)
    HIP_OK(hipEventElapsedTime(&b, ev[1], ev[2]));  // point kernel
    HIP_OK(hipEventElapsedTime(&c, ev[2], ev[3]));  // cost sum + all-reduce join
    h->bench_jac_ms += b;
    h->bench_asm_ms += a + c;
    h->bench_count++;
    if (h->bench_pair_rec[i]) {
      float d = 0.f;
      HIP_OK(hipEventElapsedTime(&d, ev[4], ev[5]));  // pair-major camera kernel
      h->bench_pair_ms += d;
      h->bench_pair_count++;
    }
  }
  h->bench_pending = 0;
  return 0;
}

extern "C" int dab_bench_eval_pass(dab_handle* h, int with_assembly, int count) {
  clear_error();
  if (!h || !h->have_problem) return set_error(DAB_E_STATE, "no problem set");
  if (count < 0) return set_error(DAB_E_INVALID, "negative pass count");
  HIP_OK(hipSetDevice(h->device));
  hipStream_t s = h->stream;
  // Timing events bracket every 8th pass (Knobs::bench_sample) of the batch (the first one always):
  // even fence-free, four event records add ~10 us to a ~40 us pass, so timing every pass
  // would distort the throughput it measures. DAB_BENCH_SAMPLE overrides (0 = no events).
  const int sample = h->knobs.bench_sample;
  for (int step = 0; step < count; ++step) {
    // every bench pass is an evaluation at a NEW linearization point, as in the LM loop
    // after an accepted step (sfm.cc:66-73, Ceres re-linearises each iteration): the pass
    // derives nothing from the points that it could keep between passes (no camera-major
    // point copy; the tables are built inside the launch)
    if (sample <= 0 || step % sample != 0) {
      CHECK_RC(eval_pass(h, false));
      CHECK_RC(h->allreduce_cost());
      continue;
    }
    // per-step events from a pool: nothing here waits for the device, so back-to-back
    // steps queue like the solver's own passes; dab_bench_kernel_ms reads them afterwards
    if (h->bench_pending >= (int)h->bench_ev.size()) {
      if (h->bench_pending >= 4096) CHECK_RC(collect_bench_events(h));
      while ((int)h->bench_ev.size() <= h->bench_pending) {
        std::array<hipEvent_t, 6> e{};
        // timing-only events: no system-scope fence (it costs several us per record)
        for (auto& x : e) HIP_OK(hipEventCreateWithFlags(&x, hipEventDisableSystemFence));
        h->bench_ev.push_back(e);
      }
    }
    h->bench_pair_rec.resize(h->bench_ev.size());
    const int slot = h->bench_pending++;
    const auto& ev = h->bench_ev[slot];
    h->bench_pair_rec[slot] = 0;
    HIP_OK(hipEventRecord(ev[0], s));
    if (with_assembly) {
      bool prec = false;
      CHECK_RC(eval_pass(h, false, ev[1], ev[2], ev[4], ev[5], &prec));
      h->bench_pair_rec[slot] = prec;
      CHECK_RC(h->allreduce_cost());
    } else {
      if (eval_points_needs_camtab(h->eval_wps)) launch_cam_tables(s, h->E, h->d_ext, h->d_camtab);
      HIP_OK(hipEventRecord(ev[1], s));
      if (eval_points_fx(h->eval_wps)) h->fx_last ^= 1;
      h->cost_fx_pending = eval_points_fx(h->eval_wps);
      launch_eval_points(s, h->view, h->d_points, h->d_ext, h->d_camtab, h->d_V, h->d_g, h->d_gpart, h->d_arrivals,
                         h->d_scal + S_COST, h->cost_fx(h->fx_last), h->cost_fx(h->fx_last ^ 1), h->eval_grid,
                         h->eval_wps);
      HIP_OK(hipEventRecord(ev[2], s));
    }
    HIP_OK(hipEventRecord(ev[3], s));
  }
  return 0;
}

extern "C" int dab_sync(dab_handle* h) {
  clear_error();
  if (!h) return set_error(DAB_E_INVALID, "null handle");
  HIP_OK(hipSetDevice(h->device));
  HIP_OK(hipStreamSynchronize(h->stream));
  if (h->d_scal) {
    HIP_OK(hipMemcpy(h->h_scal + S_XERR, h->d_scal + S_XERR, sizeof(double), hipMemcpyDeviceToHost));
    CHECK_RC(xerr_check_sticky(h));
  }
  return 0;
}

extern "C" int dab_bench_kernel_ms(dab_handle* h, double* jac_ms, double* assembly_ms) {
  clear_error();
  if (!h) return set_error(DAB_E_INVALID, "null handle");
  CHECK_RC(collect_bench_events(h));
  const double n = h->bench_count > 0 ? h->bench_count : 1;
  if (jac_ms) *jac_ms = h->bench_jac_ms / n;
  if (assembly_ms) *assembly_ms = h->bench_asm_ms / n;
  h->last_pair_ms = h->bench_pair_count > 0 ? h->bench_pair_ms / h->bench_pair_count : 0.0;
  h->bench_jac_ms = h->bench_asm_ms = h->bench_pair_ms = 0;
  h->bench_count = h->bench_pair_count = 0;
  return 0;
}

extern "C" int dab_bench_pair_ms(dab_handle* h, double* ms, double* bytes) {
  clear_error();
  if (!h || !h->have_problem) return set_error(DAB_E_STATE, "no problem set");
  // Algorithmic bytes of one k_eval_pair launch (the rig's composed observations whose two
  // cameras are free, pair-major): per observation the 16-B pixel and three index words
  // (point, arc, ring; the intrinsic is the arc's), the 24-B point once per distinct point
  // the pass touches, and per chunk its 90 sums out (two camera halves + the cross block).
  // The point array is read, in this order, by random gathers.
  if (ms) *ms = h->last_pair_ms;
  if (bytes) *bytes = h->pair_eval ? h->pair_bytes : 0.0;
  return 0;
}

extern "C" int dab_jacobian_bytes(dab_handle* h, double* bytes) {
  clear_error();
  if (!h || !h->have_problem) return set_error(DAB_E_STATE, "no problem set");
  // Algorithmic bytes of one launch of the point-side evaluation kernel (k_eval_points,
  // matrix-free residual + Jacobian reduced into V, g): the SURVEY §8d input terms
  // (16 xy + 4 n_idx per observation, n_idx = 2 single / 3 arc∘ring; 24 per point,
  // 48 per intrinsic, 48 per extrinsic) plus the outputs V, g per point (72 B). The
  // LDS variants build R, t from the 48-B extrinsics; the global-table variants read the
  // 96-B R, t part of the camera tables instead. The Jacobian itself never reaches HBM, so
  // its 16 k bytes per observation are not counted (they are not moved).
  // The fused pass (k_eval_bal) also produces the camera side: it writes U | g_c (216 B
  // per free camera) and reads every entry a second time in camera-major order (20 B:
  // point index + pixel; the chunk's camera and intrinsic are per block). A deterministic
  // matrix-free pass needs both traversal orders (point-major for V, g; camera-major for
  // U, g_c: no atomics, no per-observation partials), so both reads are algorithmic.
  // This is the minimal count whatever the implementation reads: no denormalised copies, no
  // re-gathers of a point, each traversal's index words once.
  double b = (24.0 + 72.0) * h->NP + 48.0 * h->E + 48.0 * h->NI;
  if (h->fused) b += 216.0 * h->NC + 20.0 * h->NE;
  for (int o = 0; o < h->N; ++o) b += 16.0 + 4.0 * (h->prob.obs_ext1[o] >= 0 ? 3 : 2);
  *bytes = b;
  return 0;
}

extern "C" int dab_comm_schedule(dab_handle* h, int32_t* p2p) {
  clear_error();
  if (!h || !p2p) return set_error(DAB_E_INVALID, "null argument");
  *p2p = (h->p2p_main || h->p2p_comm) ? 1 : 0;
  return 0;
}

extern "C" int dab_pcg_schedule(dab_handle* h, int32_t* matrix_free) {
  clear_error();
  if (!h || !h->have_problem || !matrix_free) return set_error(DAB_E_STATE, "no problem set");
  *matrix_free = h->pcg_built && h->mf ? (h->mf32 ? 2 : 1) : 0;
  return 0;
}

extern "C" int dab_eval_schedule(dab_handle* h, int32_t* fused) {
  clear_error();
  if (!h || !h->have_problem || !fused) return set_error(DAB_E_STATE, "no problem set");
  *fused = h->fused ? (h->fused_split ? 2 : 1) : 0;
  return 0;
}
