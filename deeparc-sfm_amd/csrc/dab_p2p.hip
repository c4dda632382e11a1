// dab_p2p.hip — one-shot peer-to-peer all-reduce over xGMI for the small camera-sized
// vectors of the multi-GPU solve (the per-CG-iteration 6 NC vector is 48 KB at
// C3, the per-pass camera blocks 216 KB; a ring all-reduce of that size is bound by its
// 2 (N - 1) latency steps, not by bandwidth).
//
// Every rank owns one region of uncached device memory (coherent across devices, so no
// cache maintenance is needed between a store on one GPU and a load on another): two data
// slots and, per slot, a flag word per (work-group, source rank). The region's IPC handle is
// exchanged once; each rank maps every peer's region. One call, with sequence number seq
// (identical on every rank: the calls of a handle are issued in the same order everywhere)
// and slot seq & 1:
//   1. work-group j copies its slice of the vector into its own region's slot;
//   2. it publishes the slice: system-scope release fence, then the flag (j, rank) := seq
//      written into every rank's region (remote vector stores over xGMI);
//   3. it waits until its own region holds flag (j, r) = seq for every rank r;
//   4. it sums slice j over the ranks' slots in rank order 0..N-1 (remote loads) into the
//      output — the same order on every rank, so every rank gets bitwise the same result.
// A slot is rewritten two calls later; by then every peer has signalled the call in
// between, which it does only after its kernel of this call (same stream) has finished
// reading. The waits are bounded (s_memrealtime deadline): a peer that never arrives sets
// the context's error word (host-pinned) instead of hanging the GPU, the call writes
// poison (NaN / all-ones / set flags) instead of a sum, and every later call of the
// context fails at once without publishing, so the peers give up too. The solver polls the
// word at every host synchronisation (p2p_check) and returns DAB_E_COMM.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "dab_internal.h"
#include "dab_p2p.h"

namespace dab {

namespace {
constexpr int kP2pBlock = 256;
// default bound of a wait for a peer: 60 s of the 100-MHz s_memrealtime clock (a peer may
// legitimately be late by its own host-side set-up; DAB_P2P_TIMEOUT_MS overrides)
constexpr long long kDefaultTimeoutMs = 60000;

struct Layout {
  size_t cap;  // 8-byte words per slot
  __host__ __device__ size_t slot_off(int s) const { return (size_t)s * cap; }
  __host__ __device__ size_t flag_off() const { return 2 * cap; }  // [2][kP2pMaxWg][kP2pMaxRanks] words
  __host__ __device__ size_t words() const { return flag_off() + 2 * (size_t)kP2pMaxWg * kP2pMaxRanks; }
};

struct PeerPtrs {
  unsigned long long* p[kP2pMaxRanks];
};

// Slot stores and loads are relaxed system-scope atomics (8-byte words): they bypass every
// non-coherent cache on both sides, whatever memory type the importing process's mapping of
// a peer region got, so a slot reused two calls later is never read from a stale line.
// 4-byte values (the flag max) travel widened to one word.
template <class T>
__device__ __forceinline__ unsigned long long to_word(T v) {
  if constexpr (sizeof(T) == 8) return __builtin_bit_cast(unsigned long long, v);
  else return (unsigned long long)__builtin_bit_cast(unsigned, v);
}
template <class T>
__device__ __forceinline__ T from_word(unsigned long long w) {
  if constexpr (sizeof(T) == 8) return __builtin_bit_cast(T, w);
  else return __builtin_bit_cast(T, (unsigned)w);
}
template <class T>
__device__ __forceinline__ void sys_store(unsigned long long* p, T v) {
  __hip_atomic_store(p, to_word(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <class T>
__device__ __forceinline__ T sys_load(const unsigned long long* p) {
  return from_word<T>(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}
// what a failed call leaves in the output: non-finite sums, all-ones cost words, set flags,
// so nothing downstream mistakes it for a result (the host sees the error word first)
template <class T>
__device__ __forceinline__ T poison() {
  if constexpr (sizeof(T) == 8 && (T)0.5 != (T)0) return __builtin_nan("");
  else return ~(T)0 > 0 ? ~(T)0 : (T)0x7fffffff;
}

// OP: 0 sum, 1 max. err: this context's error word (host-pinned, coherent): nonzero after
// a call gave up waiting; every later call then fails at once (no wait, no flag published,
// so the peers give up too) and poisons its output.
template <class T, int OP>
__global__ __launch_bounds__(kP2pBlock) void k_p2p_allreduce(T* __restrict__ buf, size_t n, size_t chunk,
                                                             PeerPtrs peers, int rank, int world, size_t cap,
                                                             unsigned long long seq, unsigned long long* err,
                                                             long long timeout_ticks) {
  const Layout L{cap};
  const int j = blockIdx.x, s = (int)(seq & 1);
  const size_t b = (size_t)j * chunk, e = b + chunk < n ? b + chunk : n;
  __shared__ int failed;
  if (threadIdx.x == 0)
    failed = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0ull ? 1 : 0;
  __syncthreads();
  if (!failed) {
    unsigned long long* mine = peers.p[rank];
    unsigned long long* my_slot = mine + L.slot_off(s);
    for (size_t i = b + threadIdx.x; i < e; i += kP2pBlock) sys_store(my_slot + i, buf[i]);
    __threadfence_system();  // the slice is visible to every device before its flag
    __syncthreads();
    if ((int)threadIdx.x < world) {
      unsigned long long* f = peers.p[threadIdx.x] + L.flag_off() + ((size_t)s * kP2pMaxWg + j) * kP2pMaxRanks + rank;
      __hip_atomic_store(f, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if ((int)threadIdx.x < world) {
      unsigned long long* f = mine + L.flag_off() + ((size_t)s * kP2pMaxWg + j) * kP2pMaxRanks + threadIdx.x;
      const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
        if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
          // give up: record the call, and publish nothing more from this context
          __hip_atomic_store(err, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          failed = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __syncthreads();
  }
  if (failed) {  // never sum slots a peer may not have written
    for (size_t i = b + threadIdx.x; i < e; i += kP2pBlock) buf[i] = poison<T>();
    return;
  }
  for (size_t i = b + threadIdx.x; i < e; i += kP2pBlock) {
    T t = sys_load<T>(peers.p[0] + L.slot_off(s) + i);
    for (int r = 1; r < world; ++r) {
      const T x = sys_load<T>(peers.p[r] + L.slot_off(s) + i);
      t = OP == 0 ? t + x : (x > t ? x : t);
    }
    buf[i] = t;
  }
}
}  // namespace

// The regions live in one process-wide arena per device, allocated and exported once and
// never freed; each peer's arena is imported once per process and never closed. A group takes
// a free slot of the arena and gives it back on destroy. Re-exporting fresh allocations per
// group was unsafe on this runtime: an importer could get back its mapping of the peer's
// earlier (freed) allocation for the new handle — two live handles of one peer were seen to
// resolve to one mapping, and on the 4-rank one-GPU rehearsal the third and later groups read
// stale slots and wrote flags into memory the peer had reused (wrong sums, then wrong
// trajectories after the fallback). With one export per process the handle an importer
// sees for a peer never changes.
namespace {
constexpr int kArenaSlots = 8;  // live groups per process and device
struct Arena {
  void* alloc = nullptr;
  size_t slot_bytes = 0;
  unsigned char rec[kP2pHandleBytes] = {};  // IPC handle | offset of the allocation in its range
  bool used[kArenaSlots] = {};
};
std::mutex g_p2p_mu;
std::map<int, Arena> g_arena;                              // device -> arena
std::map<std::pair<int, std::string>, char*> g_imported;  // (device, peer handle) -> mapping
}  // namespace

struct P2pShared {
  int device = 0, slot = -1, refs = 0;
};
struct P2pComm {
  int rank = 0, world = 1;
  size_t cap = 0;  // words per slot
  unsigned long long* mine = nullptr;
  unsigned long long* peer[kP2pMaxRanks] = {};
  unsigned long long seq = 0;
  P2pShared* shared = nullptr;
  unsigned long long* err = nullptr;  // host-pinned, coherent: the device writes, the host polls
  long long timeout_ticks = 0;        // s_memrealtime ticks (100 MHz)
  long long skip_call = 0;            // DAB_P2P_SKIP_CALL (failure-path test): this call is not launched
};

static void shared_release(P2pShared* sh) {
  if (!sh || --sh->refs > 0) return;
  if (sh->slot >= 0) {
    std::lock_guard<std::mutex> lk(g_p2p_mu);
    g_arena[sh->device].used[sh->slot] = false;
  }
  delete sh;
}

// a free slot of this device's arena (allocated and exported on first use), NOT yet zeroed:
// a peer's last call of the slot's previous group may still be reading it over its mapping.
// The device is drained first, so this rank's own calls of earlier groups are complete
// before it joins the new group's exchange; p2p_create_group zeroes the slot only after
// that exchange (every member drained), then meets the members once more before any call.
static std::string arena_take(int device, size_t bytes, int* slot, char** base, unsigned long long* soff,
                              unsigned char* rec) {
  if (hipDeviceSynchronize() != hipSuccess) return "p2p: device synchronisation failed";
  std::lock_guard<std::mutex> lk(g_p2p_mu);
  Arena& a = g_arena[device];
  if (!a.alloc) {
    void* p = nullptr;
    const size_t total = bytes * kArenaSlots;
    if (hipExtMallocWithFlags(&p, total, hipDeviceMallocUncached) != hipSuccess) return "p2p: uncached arena allocation failed";
    hipIpcMemHandle_t hd{};
    hipDeviceptr_t rbase = nullptr;
    size_t range = 0;
    if (hipIpcGetMemHandle(&hd, p) != hipSuccess || hipMemGetAddressRange(&rbase, &range, p) != hipSuccess) {
      (void)hipFree(p);
      return "p2p: arena export failed";
    }
    const unsigned long long off = (unsigned long long)(static_cast<char*>(p) - static_cast<char*>(rbase));
    a.alloc = p;
    a.slot_bytes = bytes;
    std::memcpy(a.rec, &hd, sizeof(hd));
    std::memcpy(a.rec + sizeof(hd), &off, 8);
  }
  if (bytes > a.slot_bytes) return "p2p: group larger than the arena slot";
  int k = 0;
  while (k < kArenaSlots && a.used[k]) ++k;
  if (k == kArenaSlots) return "p2p: every arena slot is in use";
  a.used[k] = true;
  *slot = k;
  *base = static_cast<char*>(a.alloc) + (size_t)k * a.slot_bytes;
  *soff = (unsigned long long)k * a.slot_bytes;
  std::memcpy(rec, a.rec, kP2pHandleBytes);
  return "";
}

// the mapping of a peer's arena, opened once per process
static char* arena_import(int device, const unsigned char* rec) {
  std::lock_guard<std::mutex> lk(g_p2p_mu);
  const auto key = std::make_pair(device, std::string(reinterpret_cast<const char*>(rec), sizeof(hipIpcMemHandle_t)));
  auto it = g_imported.find(key);
  if (it != g_imported.end()) return it->second;
  hipIpcMemHandle_t ph;
  std::memcpy(&ph, rec, sizeof(ph));
  void* q = nullptr;
  if (hipIpcOpenMemHandle(&q, ph, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return nullptr;
  char* m = static_cast<char*>(q);
  g_imported[key] = m;
  return m;
}

int p2p_create_group(int rank, int world, size_t cap_words, int nctx, const P2pAllgather& allgather,
                     P2pComm** out) {
  for (int k = 0; k < nctx; ++k) out[k] = nullptr;
  if (world < 2 || world > kP2pMaxRanks) return set_error(DAB_E_INVALID, "p2p: world size out of range");
  const Layout L{cap_words};
  const size_t region = (L.words() + 511) / 512 * 512;  // words per context, 4-KB aligned
  int device = 0;
  (void)hipGetDevice(&device);
  P2pShared* sh = new P2pShared();
  sh->device = device;
  // local failures still take part in the (collective) handle exchange, with a zero record
  char* mine = nullptr;
  unsigned char rec[kP2pHandleBytes] = {};
  unsigned long long soff = 0;
  std::string err = arena_take(device, region * nctx * 8, &sh->slot, &mine, &soff, rec);
  sh->refs = 1;
  static_assert(sizeof(hipIpcMemHandle_t) + 17 <= kP2pHandleBytes, "IPC handle size");
  // record: IPC handle | allocation offset in its range (8) | slot offset in the arena (8) | valid
  std::vector<unsigned char> all((size_t)world * kP2pHandleBytes, 0);
  if (err.empty()) {
    unsigned char* r = all.data() + (size_t)rank * kP2pHandleBytes;
    std::memcpy(r, rec, sizeof(hipIpcMemHandle_t) + 8);
    std::memcpy(r + sizeof(hipIpcMemHandle_t) + 8, &soff, 8);
    r[sizeof(hipIpcMemHandle_t) + 16] = 1;  // valid record
  }
  if (allgather(all.data()) != 0) {
    shared_release(sh);
    return set_error(DAB_E_COMM, "p2p: handle exchange failed");
  }
  // Every member drained its device before the exchange, so no call of an earlier group
  // still reads this rank's slot: zero it now (stale flags and data), then meet once more
  // (a second exchange of one status byte each) so that no member publishes into the slot
  // before it is clear. Both exchanges run on every rank, whatever failed locally.
  if (err.empty() && (hipMemset(mine, 0, region * nctx * 8) != hipSuccess || hipDeviceSynchronize() != hipSuccess))
    err = "p2p: arena slot initialisation failed";
  std::vector<unsigned char> ok((size_t)world * kP2pHandleBytes, 0);
  ok[(size_t)rank * kP2pHandleBytes] = err.empty() ? 1 : 0;
  if (allgather(ok.data()) != 0) {
    shared_release(sh);
    return set_error(DAB_E_COMM, "p2p: handle exchange failed");
  }
  for (int r = 0; r < world && err.empty(); ++r) {
    if (all[(size_t)r * kP2pHandleBytes + sizeof(hipIpcMemHandle_t) + 16] != 1) err = "p2p: a peer could not export its region";
    else if (ok[(size_t)r * kP2pHandleBytes] != 1) err = "p2p: a peer could not initialise its region";
  }
  if (!err.empty()) {
    shared_release(sh);
    return set_error(DAB_E_DEVICE, err);
  }
  std::vector<char*> peer_base(world, nullptr);
  for (int r = 0; r < world; ++r) {
    if (r == rank) {
      peer_base[r] = mine;
      continue;
    }
    const unsigned char* pr = all.data() + (size_t)r * kP2pHandleBytes;
    unsigned long long poff = 0, psoff = 0;
    std::memcpy(&poff, pr + sizeof(hipIpcMemHandle_t), 8);
    std::memcpy(&psoff, pr + sizeof(hipIpcMemHandle_t) + 8, 8);
    char* q = arena_import(device, pr);
    if (!q) {
      shared_release(sh);
      return set_error(DAB_E_DEVICE, "p2p: hipIpcOpenMemHandle failed");
    }
    peer_base[r] = q + poff + psoff;
  }
  sh->refs = nctx;
  long long tmo_ms = kDefaultTimeoutMs, skip = 0;
  if (const char* e = getenv("DAB_P2P_TIMEOUT_MS")) tmo_ms = std::max(1LL, atoll(e));
  if (const char* e = getenv("DAB_P2P_SKIP_CALL")) skip = atoll(e);
  for (int k = 0; k < nctx; ++k) {
    P2pComm* c = new P2pComm();
    c->rank = rank;
    c->world = world;
    c->cap = cap_words;
    c->shared = sh;
    for (int r = 0; r < world; ++r)
      c->peer[r] = reinterpret_cast<unsigned long long*>(peer_base[r]) + (size_t)k * region;
    c->mine = c->peer[rank];
    c->timeout_ticks = tmo_ms * 100000LL;
    c->skip_call = k == 0 ? skip : 0;
    void* e = nullptr;
    if (hipHostMalloc(&e, 64, hipHostMallocCoherent) != hipSuccess) {
      sh->refs = k + 1;  // the contexts made so far hold the slot: destroying them returns it
      for (int q = 0; q <= k; ++q) p2p_destroy(q < k ? out[q] : c);
      for (int q = 0; q < nctx; ++q) out[q] = nullptr;
      return set_error(DAB_E_NOMEM, "p2p: pinned error word allocation failed");
    }
    c->err = static_cast<unsigned long long*>(e);
    *c->err = 0;
    out[k] = c;
  }
  return 0;
}

void p2p_destroy(P2pComm* c) {
  if (!c) return;
  shared_release(c->shared);
  if (c->err) (void)hipHostFree(c->err);
  delete c;
}

size_t p2p_capacity(const P2pComm* c) { return c ? c->cap : 0; }

template <class T, int OP>
static int p2p_reduce(P2pComm* c, hipStream_t s, T* buf, size_t n) {
  if (n > c->cap) return set_error(DAB_E_INVALID, "p2p: vector larger than the slot");
  if (n == 0) return 0;
  // slices of >= 2048 words; at most kP2pMaxWg work-groups, each reading its slice from
  // every peer (the xGMI links are point to point, so every peer is read in parallel)
  const size_t chunk = std::max<size_t>(2048, (n + kP2pMaxWg - 1) / kP2pMaxWg);
  const int grid = (int)((n + chunk - 1) / chunk);
  PeerPtrs pp{};
  for (int r = 0; r < c->world; ++r) pp.p[r] = c->peer[r];
  ++c->seq;
  if ((long long)c->seq == c->skip_call) return 0;  // failure-path test: this rank misses one call
  k_p2p_allreduce<T, OP><<<grid, kP2pBlock, 0, s>>>(buf, n, chunk, pp, c->rank, c->world, c->cap, c->seq, c->err,
                                                    c->timeout_ticks);
  return hipGetLastError() == hipSuccess ? 0 : set_error(DAB_E_DEVICE, "p2p: launch failed");
}
int p2p_allreduce_sum(P2pComm* c, hipStream_t s, double* buf, size_t n) { return p2p_reduce<double, 0>(c, s, buf, n); }
int p2p_allreduce_sum_u64(P2pComm* c, hipStream_t s, unsigned long long* buf, size_t n) {
  return p2p_reduce<unsigned long long, 0>(c, s, buf, n);
}
int p2p_allreduce_max(P2pComm* c, hipStream_t s, double* buf, size_t n) { return p2p_reduce<double, 1>(c, s, buf, n); }
int p2p_allreduce_max_i32(P2pComm* c, hipStream_t s, int* buf, size_t n) { return p2p_reduce<int, 1>(c, s, buf, n); }

// One verified exchange before the path is trusted: two sums (both slots of the context)
// of known integer patterns, exact in fp64, under a short timeout. A peer mapping that
// does not deliver (a platform where the IPC-mapped uncached region is not coherent across
// devices, say) shows up here, at set-up, and the caller keeps RCCL instead.
int p2p_selftest(P2pComm* c, hipStream_t s) {
  const size_t n = std::min<size_t>(c->cap, 4096);  // two work-groups' slices
  if (n == 0) return 0;
  const long long keep = c->timeout_ticks;
  c->timeout_ticks = std::min<long long>(keep, 3000LL * 100000LL);  // 3 s
  double* d = nullptr;
  if (hipMalloc(&d, n * sizeof(double)) != hipSuccess) {
    c->timeout_ticks = keep;
    return set_error(DAB_E_NOMEM, "p2p self-test: allocation failed");
  }
  std::vector<double> h(n);
  int rc = 0;
  const double w = (double)c->world, tri = w * (w + 1.0) / 2.0;
  // DAB_P2P_SELFTEST_SKEW=r (test knob): rank r contributes a wrong word, so every rank's
  // check fails and the set-up falls back
  const char* sk = getenv("DAB_P2P_SELFTEST_SKEW");
  const bool skew = sk && atoi(sk) == c->rank;
  for (int call = 0; call < 2 && rc == 0; ++call) {
    for (size_t k = 0; k < n; ++k) h[k] = (double)(c->rank + 1) * (double)(k + 1 + call);
    if (skew) h[0] += 1.0;
    if (hipMemcpy(d, h.data(), n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
        p2p_allreduce_sum(c, s, d, n) != 0 || hipStreamSynchronize(s) != hipSuccess ||
        hipMemcpy(h.data(), d, n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) {
      rc = set_error(DAB_E_DEVICE, "p2p self-test: a call failed");
      break;
    }
    if (p2p_check(c) != 0) {
      rc = -1;
      break;
    }
    for (size_t k = 0; k < n; ++k)
      if (h[k] != tri * (double)(k + 1 + call)) {
        rc = set_error(DAB_E_COMM, "p2p self-test: wrong sum at word " + std::to_string(k));
        break;
      }
  }
  (void)hipFree(d);
  c->timeout_ticks = keep;
  return rc;
}

int p2p_check(P2pComm* c) {
  if (!c || !c->err) return 0;
  const unsigned long long e = __atomic_load_n(c->err, __ATOMIC_ACQUIRE);
  if (e != 0) return set_error(DAB_E_COMM, "p2p all-reduce: a peer did not arrive (call " + std::to_string(e) + ")");
  return 0;
}

// Loads this translation unit's code object on the current device now: otherwise the first
// launch of any of its kernels pays for it (10-40 ms, inside a process's first LM iteration).
void warm_p2p() {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(k_p2p_allreduce<double, 0>));
}

}  // namespace dab
