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
// reading. The waits are bounded: a peer that never arrives sets the region's error word
// instead of hanging the GPU (p2p_check reports it).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "dab_internal.h"
#include "dab_p2p.h"

namespace dab {

namespace {
constexpr int kP2pBlock = 256;
constexpr size_t kSpinLimit = size_t(1) << 26;  // ~1 s of polling before giving up

struct Layout {
  size_t cap;  // 8-byte words per slot
  __host__ __device__ size_t slot_off(int s) const { return (size_t)s * cap; }
  __host__ __device__ size_t flag_off() const { return 2 * cap; }  // [2][kP2pMaxWg][kP2pMaxRanks] words
  __host__ __device__ size_t err_off() const { return flag_off() + 2 * (size_t)kP2pMaxWg * kP2pMaxRanks; }
  __host__ __device__ size_t words() const { return err_off() + 16; }
};

struct PeerPtrs {
  unsigned long long* p[kP2pMaxRanks];
};

// Slot stores and loads are relaxed system-scope atomics (8-byte words): they bypass every
// non-coherent cache on both sides, whatever memory type the importing process's mapping of
// a peer region got, so a slot reused two calls later is never read from a stale line.
template <class T>
__device__ __forceinline__ void sys_store(T* p, T v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <class T>
__device__ __forceinline__ T sys_load(const T* p) {
  return __builtin_bit_cast(T, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_SYSTEM));
}

template <class T>
__global__ __launch_bounds__(kP2pBlock) void k_p2p_allreduce(T* __restrict__ buf, size_t n, size_t chunk,
                                                             PeerPtrs peers, int rank, int world, size_t cap,
                                                             unsigned long long seq) {
  const Layout L{cap};
  const int j = blockIdx.x, s = (int)(seq & 1);
  const size_t b = (size_t)j * chunk, e = b + chunk < n ? b + chunk : n;
  unsigned long long* mine = peers.p[rank];
  T* my_slot = reinterpret_cast<T*>(mine + L.slot_off(s));
  for (size_t i = b + threadIdx.x; i < e; i += kP2pBlock) sys_store(my_slot + i, buf[i]);
  __threadfence_system();  // the slice is visible to every device before its flag
  __syncthreads();
  if ((int)threadIdx.x < world) {
    unsigned long long* f = peers.p[threadIdx.x] + L.flag_off() + ((size_t)s * kP2pMaxWg + j) * kP2pMaxRanks + rank;
    __hip_atomic_store(f, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if ((int)threadIdx.x < world) {
    unsigned long long* f = mine + L.flag_off() + ((size_t)s * kP2pMaxWg + j) * kP2pMaxRanks + threadIdx.x;
    size_t spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
      if (++spins > kSpinLimit) {
        __hip_atomic_store(mine + L.err_off(), seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  for (size_t i = b + threadIdx.x; i < e; i += kP2pBlock) {
    T t = sys_load(reinterpret_cast<const T*>(peers.p[0] + L.slot_off(s)) + i);
    for (int r = 1; r < world; ++r) t += sys_load(reinterpret_cast<const T*>(peers.p[r] + L.slot_off(s)) + i);
    buf[i] = t;
  }
}
}  // namespace

// One allocation per rank holds the regions of every context of a group (each process
// opens each peer's handle once: two handles of one peer opened in one process were seen
// to resolve to the same mapping on the one-GPU rehearsal).
struct P2pShared {
  int rank = 0, world = 1, refs = 0;
  void* alloc = nullptr;
  void* opened[kP2pMaxRanks] = {};  // what hipIpcOpenMemHandle returned (closed on release)
};
struct P2pComm {
  int rank = 0, world = 1;
  size_t cap = 0;  // words per slot
  unsigned long long* mine = nullptr;
  unsigned long long* peer[kP2pMaxRanks] = {};
  unsigned long long seq = 0;
  P2pShared* shared = nullptr;
};

static void shared_release(P2pShared* sh) {
  if (!sh || --sh->refs > 0) return;
  for (int r = 0; r < sh->world; ++r)
    if (r != sh->rank && sh->opened[r]) (void)hipIpcCloseMemHandle(sh->opened[r]);
  if (sh->alloc) (void)hipFree(sh->alloc);
  delete sh;
}

int p2p_create_group(int rank, int world, size_t cap_words, int nctx, const P2pAllgather& allgather,
                     P2pComm** out) {
  for (int k = 0; k < nctx; ++k) out[k] = nullptr;
  if (world < 2 || world > kP2pMaxRanks) return set_error(DAB_E_INVALID, "p2p: world size out of range");
  const Layout L{cap_words};
  const size_t region = (L.words() + 511) / 512 * 512;  // words per context, 4-KB aligned
  P2pShared* sh = new P2pShared();
  sh->rank = rank;
  sh->world = world;
  // local failures still take part in the (collective) handle exchange, with a zero record
  std::string err;
  void* p = nullptr;
  hipIpcMemHandle_t hd{};
  unsigned long long off = 0;
  if (hipExtMallocWithFlags(&p, region * nctx * 8, hipDeviceMallocUncached) != hipSuccess) {
    p = nullptr;
    err = "p2p: uncached region allocation failed";
  } else {
    sh->alloc = p;
    hipDeviceptr_t base = nullptr;  // the handle names the whole allocation: send the offset too
    size_t range = 0;
    if (hipMemset(p, 0, region * nctx * 8) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
      err = "p2p: region initialisation failed";
    else if (hipIpcGetMemHandle(&hd, p) != hipSuccess)
      err = "p2p: hipIpcGetMemHandle failed";
    else if (hipMemGetAddressRange(&base, &range, p) != hipSuccess)
      err = "p2p: hipMemGetAddressRange failed";
    else
      off = (unsigned long long)(static_cast<char*>(p) - static_cast<char*>(base));
  }
  sh->refs = 1;
  static_assert(sizeof(hipIpcMemHandle_t) + 9 <= kP2pHandleBytes, "IPC handle size");
  std::vector<unsigned char> all((size_t)world * kP2pHandleBytes, 0);
  if (err.empty()) {
    std::memcpy(all.data() + (size_t)rank * kP2pHandleBytes, &hd, sizeof(hd));
    std::memcpy(all.data() + (size_t)rank * kP2pHandleBytes + sizeof(hd), &off, 8);
    all[(size_t)rank * kP2pHandleBytes + sizeof(hd) + 8] = 1;  // valid record
  }
  if (allgather(all.data()) != 0) {
    shared_release(sh);
    return set_error(DAB_E_COMM, "p2p: handle exchange failed");
  }
  for (int r = 0; r < world && err.empty(); ++r)
    if (all[(size_t)r * kP2pHandleBytes + sizeof(hd) + 8] != 1) err = "p2p: a peer could not export its region";
  if (!err.empty()) {
    shared_release(sh);
    return set_error(DAB_E_DEVICE, err);
  }
  std::vector<char*> peer_base(world, nullptr);
  for (int r = 0; r < world; ++r) {
    if (r == rank) {
      peer_base[r] = static_cast<char*>(p);
      continue;
    }
    hipIpcMemHandle_t ph;
    unsigned long long poff = 0;
    std::memcpy(&ph, all.data() + (size_t)r * kP2pHandleBytes, sizeof(ph));
    std::memcpy(&poff, all.data() + (size_t)r * kP2pHandleBytes + sizeof(ph), 8);
    void* q = nullptr;
    if (hipIpcOpenMemHandle(&q, ph, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      shared_release(sh);
      return set_error(DAB_E_DEVICE, "p2p: hipIpcOpenMemHandle failed");
    }
    sh->opened[r] = q;
    peer_base[r] = static_cast<char*>(q) + poff;
  }
  sh->refs = nctx;
  for (int k = 0; k < nctx; ++k) {
    P2pComm* c = new P2pComm();
    c->rank = rank;
    c->world = world;
    c->cap = cap_words;
    c->shared = sh;
    for (int r = 0; r < world; ++r)
      c->peer[r] = reinterpret_cast<unsigned long long*>(peer_base[r]) + (size_t)k * region;
    c->mine = c->peer[rank];
    out[k] = c;
  }
  return 0;
}

void p2p_destroy(P2pComm* c) {
  if (!c) return;
  shared_release(c->shared);
  delete c;
}

size_t p2p_capacity(const P2pComm* c) { return c ? c->cap : 0; }

template <class T>
static int p2p_sum(P2pComm* c, hipStream_t s, T* buf, size_t n) {
  if (n > c->cap) return set_error(DAB_E_INVALID, "p2p: vector larger than the slot");
  if (n == 0) return 0;
  // slices of >= 2048 words; at most kP2pMaxWg work-groups, each reading its slice from
  // every peer (the xGMI links are point to point, so every peer is read in parallel)
  const size_t chunk = std::max<size_t>(2048, (n + kP2pMaxWg - 1) / kP2pMaxWg);
  const int grid = (int)((n + chunk - 1) / chunk);
  PeerPtrs pp{};
  for (int r = 0; r < c->world; ++r) pp.p[r] = c->peer[r];
  ++c->seq;
  k_p2p_allreduce<T><<<grid, kP2pBlock, 0, s>>>(buf, n, chunk, pp, c->rank, c->world, c->cap, c->seq);
  return hipGetLastError() == hipSuccess ? 0 : set_error(DAB_E_DEVICE, "p2p: launch failed");
}
int p2p_allreduce_sum(P2pComm* c, hipStream_t s, double* buf, size_t n) { return p2p_sum(c, s, buf, n); }
int p2p_allreduce_sum_u64(P2pComm* c, hipStream_t s, unsigned long long* buf, size_t n) {
  return p2p_sum(c, s, buf, n);
}

int p2p_check(P2pComm* c) {
  if (!c) return 0;
  unsigned long long e = 0;
  const Layout L{c->cap};
  if (hipMemcpy(&e, c->mine + L.err_off(), 8, hipMemcpyDeviceToHost) != hipSuccess)
    return set_error(DAB_E_DEVICE, "p2p: error word read failed");
  if (e != 0) return set_error(DAB_E_COMM, "p2p all-reduce: a peer did not arrive (call " + std::to_string(e) + ")");
  return 0;
}

}  // namespace dab
