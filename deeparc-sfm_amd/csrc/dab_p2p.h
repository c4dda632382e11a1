// dab_p2p.h — one-shot peer-to-peer all-reduce over xGMI (dab_p2p.hip). Internal, not ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <functional>

namespace dab {

constexpr int kP2pMaxRanks = 8;    // one node
constexpr int kP2pMaxWg = 32;      // work-groups (slices) per call
constexpr int kP2pHandleBytes = 96;  // IPC handle (64) | allocation offset (8) | arena slot offset (8) | valid

struct P2pComm;
// in-place gather of every rank's kP2pHandleBytes record: buf[world][kP2pHandleBytes], own
// row filled, the others zero on entry; 0 on success
using P2pAllgather = std::function<int(unsigned char* buf)>;

// nctx contexts (one per stream that issues sums) over one allocation and one handle
// exchange; cap_words: the largest vector (8-byte words) one call reduces
int p2p_create_group(int rank, int world, size_t cap_words, int nctx, const P2pAllgather& allgather,
                     P2pComm** out);
void p2p_destroy(P2pComm* c);
size_t p2p_capacity(const P2pComm* c);
// in-place sum over the ranks, enqueued on s (every rank calls in the same order)
int p2p_allreduce_sum(P2pComm* c, hipStream_t s, double* buf, size_t n);
int p2p_allreduce_sum_u64(P2pComm* c, hipStream_t s, unsigned long long* buf, size_t n);
// in-place max over the ranks
int p2p_allreduce_max(P2pComm* c, hipStream_t s, double* buf, size_t n);
int p2p_allreduce_max_i32(P2pComm* c, hipStream_t s, int* buf, size_t n);
// DAB_E_COMM when a call gave up waiting for a peer: a host read of the pinned error word,
// no device synchronisation (call it after the stream has drained to cover every call)
int p2p_check(P2pComm* c);
// two verified sums on the context (3-s timeout); 0 when the path delivers exact results
int p2p_selftest(P2pComm* c, hipStream_t s);

}  // namespace dab
