// dab_devmem.h — the library's device allocator (not part of the ABI).
//
// Every device buffer of a handle comes from a Dev: the problem's buffers (released into a
// pool by the next dab_set_problem and reused by best fit), the buffers kept across set-ups
// (dense S, the camera step) and the Cholesky's scratch (block inverses, ready flags, the
// grid-barrier word). One allocator means one memory-safety net for all of them:
//   DAB_DEV_GUARD=1   a 64-KB zero canary after every block; guard_check() reports the first
//                     block whose canary holds a nonzero byte, and the entry points fail
//                     closed on it (DAB_E_DEVICE, the block named in dab_last_error)
//   DAB_DEV_POISON=1  every block handed out is filled with 0xFF bytes (NaN doubles), so a
//                     read of memory nobody wrote shows; =2 fills 0x41 (finite doubles)
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "dab_internal.h"

namespace dab {

struct Dev {
  struct Blk {
    void* p;
    size_t bytes;
    int age;
    bool slab;  // carved from a slab: never freed on its own
  };
  explicit Dev(const char* name_ = "problem buffers") : name(name_) {}
  Dev(const Dev&) = delete;
  Dev& operator=(const Dev&) = delete;
  const char* name;  // named in guard reports
  std::vector<Blk> live, pool, spare;  // spare: slab pieces aged out of the pool
  // Blocks up to kSmall come from 8 MB slabs (bump-allocated). DAB_DEV_SLAB=1 turns the slabs
  // on (off by default: it did not shorten a handle's destruction)
  static constexpr size_t kSlab = (size_t)8 << 20;
  const size_t kSmall = getenv("DAB_DEV_SLAB") && atoi(getenv("DAB_DEV_SLAB")) != 0 ? (size_t)1 << 20 : 0;
  std::vector<void*> slabs;
  size_t slab_off = kSlab;
  // other allocators of the same handle whose pooled (idle) blocks are given back to the
  // device when an allocation here fails, before the one retry
  std::vector<Dev*> donors;
  ~Dev() { clear(); }
  void clear() {  // free everything now, pooled blocks included
    for (const Blk& b : live)
      if (!b.slab) (void)hipFree(b.p);
    for (const Blk& b : pool)
      if (!b.slab) (void)hipFree(b.p);
    for (void* q : slabs) (void)hipFree(q);
    live.clear();
    pool.clear();
    spare.clear();
    slabs.clear();
    guards.clear();
    slab_off = kSlab;
  }
  // a block's memory goes back to the device (its canaries with it)
  void free_blk(const Blk& b) {
    forget(b);
    (void)hipFree(b.p);
  }
  void forget(const Blk& b) {
    char* lo = static_cast<char*>(b.p);
    char* hi = lo + b.bytes;
    guards.erase(std::remove_if(guards.begin(), guards.end(), [&](const Guard& x) { return x.p >= lo && x.p < hi; }),
                 guards.end());
  }
  // every live block goes to the pool (the caller has synchronised the streams that use them)
  void release() {
    std::vector<Blk> keep;
    for (Blk& b : pool) {
      if (++b.age < 2) keep.push_back(b);
      else if (b.slab) spare.push_back(b);
      else free_blk(b);
    }
    for (Blk b : live) {
      b.age = 0;
      keep.push_back(b);
    }
    pool.swap(keep);
    live.clear();
  }
  // one live block back to the device now (a buffer re-sized outside the release cycle)
  void drop(void* p) {
    if (!p) return;
    for (size_t i = 0; i < live.size(); ++i)
      if (live[i].p == p) {
        forget(live[i]);
        if (live[i].slab) spare.push_back(live[i]);
        else (void)hipFree(p);
        live[i] = live.back();
        live.pop_back();
        return;
      }
  }
  // Pooled blocks beyond `keep` bytes go back to the device (largest first), so that a new
  // problem's allocations do not compete with memory the pool holds idly
  void trim_pool(size_t keep) {
    size_t held = 0;
    for (const Blk& b : pool) held += b.bytes;
    if (held <= keep) return;
    std::sort(pool.begin(), pool.end(), [](const Blk& a, const Blk& b) { return a.bytes > b.bytes; });
    std::vector<Blk> kept;
    for (const Blk& b : pool) {
      if (held > keep && !b.slab) {
        free_blk(b);
        held -= b.bytes;
      } else {
        kept.push_back(b);
      }
    }
    pool.swap(kept);
  }
  size_t pooled_bytes() const {
    size_t t = 0;
    for (const Blk& b : pool) t += b.bytes;
    return t;
  }
  // best fit in v among blocks of bytes .. cap; v.size() when none
  static size_t best_fit(const std::vector<Blk>& v, size_t bytes, size_t cap) {
    size_t best = v.size();
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i].bytes >= bytes && v[i].bytes <= cap && (best == v.size() || v[i].bytes < v[best].bytes)) best = i;
    return best;
  }
  static constexpr size_t kGuard = (size_t)64 << 10;
  struct Guard {
    char* p;       // the canary's first byte
    size_t bytes;  // the block's usable size
    int serial;
  };
  std::vector<Guard> guards;
  int serial = 0;
  static bool guard_on() { return guard_mode() != 0; }
  // 2: guard on, and the self-test of the net: guard_fail dirties one canary after each
  // dab_set_problem, which must then fail closed (tests/test_gpu_guard.py)
  static int guard_mode() {
    static const int m = getenv("DAB_DEV_GUARD") ? atoi(getenv("DAB_DEV_GUARD")) : 0;
    return m;
  }
  static bool poison_on() {
    static const bool on = getenv("DAB_DEV_POISON") && atoi(getenv("DAB_DEV_POISON")) != 0;
    return on;
  }
  static int poison_byte() {
    static const int b = getenv("DAB_DEV_POISON") && atoi(getenv("DAB_DEV_POISON")) == 2 ? 0x41 : 0xFF;
    return b;
  }
  // 0, or the number of overwritten canaries; the first one is described in *first (and every
  // one on stderr). The caller has synchronised the device.
  int guard_check(const char* where, std::string* first = nullptr) {
    int bad = 0;
    std::vector<unsigned char> h(kGuard);
    for (const Guard& g : guards) {
      if (hipMemcpy(h.data(), g.p, kGuard, hipMemcpyDeviceToHost) != hipSuccess) {
        ++bad;
        if (first && first->empty()) *first = std::string(name) + ": canary of block #" + std::to_string(g.serial) +
                                               " unreadable after " + where;
        continue;
      }
      size_t at = kGuard;
      for (size_t i = 0; i < kGuard; ++i)
        if (h[i] != 0) {
          at = i;
          break;
        }
      if (at < kGuard) {
        ++bad;
        const std::string msg = std::string(name) + ": block #" + std::to_string(g.serial) + " of " +
                                std::to_string(g.bytes) + " bytes overrun at +" + std::to_string(at) + " (after " +
                                where + ")";
        std::fprintf(stderr, "dab guard: %s\n", msg.c_str());
        if (first && first->empty()) *first = msg;
      }
    }
    return bad;
  }
  template <class T>
  int alloc(T** out, size_t n) {
    if (n == 0) n = 1;
    const size_t want = (n * sizeof(T) + 255) & ~(size_t)255;
    const size_t bytes = want + (guard_on() ? kGuard : 0);
    const size_t cap = std::max(2 * bytes, bytes + ((size_t)1 << 20));
    Blk got{nullptr, bytes, 0, false};
    for (std::vector<Blk>* v : {&pool, &spare}) {
      const size_t i = best_fit(*v, bytes, cap);
      if (i < v->size()) {
        got = (*v)[i];
        got.age = 0;
        (*v)[i] = v->back();
        v->pop_back();
        break;
      }
    }
    if (!got.p && bytes <= kSmall) {
      if (slab_off + bytes > kSlab) {
        void* q = nullptr;
        if (hipMalloc(&q, kSlab) == hipSuccess) {
          slabs.push_back(q);
          slab_off = 0;
        }
      }
      if (slab_off + bytes <= kSlab) {
        got = Blk{static_cast<char*>(slabs.back()) + slab_off, bytes, 0, true};
        slab_off += bytes;
      }
    }
    if (!got.p) {
      void* p = nullptr;
      if (hipMalloc(&p, bytes) != hipSuccess) {
        // the pools may hold what the device needs: give them back and try once more
        for (const Blk& b : pool) {
          if (b.slab) spare.push_back(b);
          else free_blk(b);
        }
        pool.clear();
        for (Dev* d : donors) d->trim_pool(0);
        if (hipMalloc(&p, bytes) != hipSuccess)
          return set_error(DAB_E_NOMEM, "hipMalloc of " + std::to_string(bytes) + " bytes failed");
      }
      got = Blk{p, bytes, 0, false};
    }
    live.push_back(got);
    *out = static_cast<T*>(got.p);
    // (the fills run on the null stream, which does not order against the handle's
    // non-blocking stream: the device is synchronised after them, or the handle's own
    // uploads could land first and be overwritten)
    if (poison_on()) (void)hipMemset(got.p, poison_byte(), want);
    if (guard_on()) {
      char* g = static_cast<char*>(got.p) + want;
      (void)hipMemset(g, 0, kGuard);  // zeros: a stray read of the canary is a harmless 0 / index 0
    }
    if (poison_on() || guard_on()) (void)hipDeviceSynchronize();
    if (guard_on()) {
      char* g = static_cast<char*>(got.p) + want;
      // a reused block drops the canaries of its earlier uses (now inside its usable bytes)
      forget(got);
      guards.push_back(Guard{g, want, serial});
    }
    ++serial;
    return 0;
  }
};

}  // namespace dab
