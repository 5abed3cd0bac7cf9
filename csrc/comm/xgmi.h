// One-shot all-reduce over xGMI peer memory for latency-bound buckets.
//
// Why: the reference's DDP toy all-reduces one 84-byte bucket per step
// (SURVEY M5); at that size RCCL's cost is pure latency (a kernel launch plus
// its protocol round trips). An 8x MI355X node is a fully connected xGMI mesh,
// so every rank can write straight into every peer's memory: one hop, no ring.
//
// Protocol (NCCL's "LL" idea, CDNA-native): each 4-byte value travels as an
// 8-byte word {seq:32 | value:32} written with ONE 64-bit system-scope store
// into slot [parity][src_rank][i] of every peer's buffer. A reader polls its
// own buffer until the word's seq matches, so data and flag arrive together:
// no __threadfence_system, no separate flag round trip. The buffer is
// allocated uncached (hipDeviceMallocUncached) and shared by IPC handles, so
// remote xGMI writes are visible to the owner's polls without L2 staleness.
// Two parities (seq & 1) make slot reuse safe: a rank can only start
// collective s+2 after it has read every peer's data of s+1, which each peer
// wrote after finishing s. Every rank sums the W contributions in rank order,
// so all ranks get bit-identical results (DDP replicas stay in sync). Polls are
// bounded: a peer that never arrives sets *err and the kernel completes (with
// garbage) instead of hanging the GPU; the host checks *err.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ptdt {

constexpr int kXgmiMaxRanks = 8;
// Poll budget per slot (~1 us per uncached round trip): a few seconds, far above
// any launch skew between ranks, far below a hang.
constexpr uint32_t kXgmiMaxPolls = 1u << 22;

struct XgmiArgs {
  uint64_t* local;                       // this rank's LL buffer
  uint64_t* peers[kXgmiMaxRanks];        // every rank's LL buffer (peers[rank] == local)
  uint32_t* seq;                         // this rank's collective counter (device)
  int* err;                              // nonzero after a timed-out poll
  int rank, world, max_elems;            // world == 0: disabled
  uint32_t max_polls;                    // poll budget per slot (kXgmiMaxPolls; PTDT_XGMI_MAX_POLLS)
  uint32_t drop_push;                    // fault injection: from collective seq drop_push on (0: never) skip
                                         // pushes to other ranks (PTDT_FAULT_XGMI_DROP_RANK / _SEQ)
  uint32_t flags;                        // kXgmiPair: the single-wave engine's packed-words exchange (world 2..8)
};
constexpr uint32_t kXgmiPair = 1u;  // PTDT_XGMI_PAIR=0 clears it (A/B against the chunked exchange)

#ifdef __HIPCC__
__device__ __forceinline__ uint64_t* xgmi_slot(uint64_t* base, int parity, int src, int world, int max_elems,
                                               int i) {
  return base + ((int64_t)(parity * world + src) * max_elems + i);
}

// Push this rank's n values (vals: any memory readable by the caller's threads).
// Peer-outer loop: no per-element division, consecutive lanes write consecutive words.
__device__ __forceinline__ void xgmi_push(const XgmiArgs& x, uint32_t s, const float* vals, int n, int tid,
                                          int nt) {
  const int parity = (int)(s & 1u);
  const uint64_t hi = (uint64_t)s << 32;
  for (int i = tid; i < n; i += nt) {
    const uint64_t w = hi | (uint64_t)__float_as_uint(vals[i]);
    for (int p = 0; p < x.world; ++p)
      if (x.drop_push == 0u || s < x.drop_push || p == x.rank)
        __hip_atomic_store(xgmi_slot(x.peers[p], parity, x.rank, x.world, x.max_elems, i), w, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Wait for element i of every rank and return the sum in rank order.
__device__ __forceinline__ float xgmi_gather_sum(const XgmiArgs& x, uint32_t s, int i) {
  const int parity = (int)(s & 1u);
  float acc = 0.f;
  bool dead = false;  // one timed-out peer: do not wait for the others again
  for (int p = 0; p < x.world; ++p) {
    uint64_t* slot = xgmi_slot(x.local, parity, p, x.world, x.max_elems, i);
    uint64_t w = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t polls = dead ? x.max_polls : 0;
    while ((uint32_t)(w >> 32) != s) {
      if (++polls > x.max_polls) {  // ~seconds: a peer is gone; fail loudly, never hang
        __hip_atomic_store(x.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        dead = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      w = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    acc += __uint_as_float((uint32_t)w);
  }
  return acc;
}
#endif

#ifdef __HIPCC__
// Poll every (rank, element) slot of elements [i0, i0+n) and stage the values
// in tmp[p * n + i]; the caller barriers, then sums in rank order. Each thread
// keeps U uncached loads in flight: one memory round trip per batch instead
// of one per slot (W * n / nt of them: ~60 us per step for a 2K-parameter
// bucket at W = 8). Slots whose word is not there yet are re-polled as a batch
// (bounded; a timed-out poll sets *x.err and *lds_flag when given). U costs
// 3 VGPRs per slot: 8 fits 1024-thread kernels, 256-thread kernels take 16.
template <int U = 8>
__device__ __forceinline__ void xgmi_gather_lds(const XgmiArgs& x, uint32_t s, int i0, int n, float* tmp,
                                                int tid, int nt, int* lds_flag = nullptr) {
  const int parity = (int)(s & 1u);
  const int tot = x.world * n;
  bool dead = false;  // after one timed-out slot this thread stops waiting: bounded total stall
  for (int e0 = tid; e0 < tot; e0 += U * nt) {
    uint64_t w[U];
    int off[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {  // issue the whole batch first
      const int e = e0 + u * nt;
      off[u] = -1;
      w[u] = 0;
      if (e < tot) {
        const int p = e / n, i = e - p * n;
        off[u] = (parity * x.world + p) * x.max_elems + i0 + i;
        w[u] = __hip_atomic_load(x.local + off[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    // re-poll every slot still missing, all of them in flight together: a slot that
    // arrives late costs one more round trip for the batch, not one per slot
    uint32_t polls = dead ? x.max_polls : 0;
    for (;;) {
      bool missing = false;
#pragma unroll
      for (int u = 0; u < U; ++u) missing |= off[u] >= 0 && (uint32_t)(w[u] >> 32) != s;
      if (!missing) break;
      if (++polls > x.max_polls) {
        __hip_atomic_store(x.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (lds_flag) *lds_flag = 1;
        dead = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (off[u] >= 0 && (uint32_t)(w[u] >> 32) != s)
          w[u] = __hip_atomic_load(x.local + off[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (off[u] >= 0) tmp[e0 + u * nt] = __uint_as_float((uint32_t)w[u]);
  }
}

// Sum staged contributions in rank order (bit-identical on every rank).
__device__ __forceinline__ float xgmi_sum_lds(const float* tmp, int world, int n, int i) {
  float acc = 0.f;
  for (int p = 0; p < world; ++p) acc += tmp[p * n + i];
  return acc;
}
#endif

// Standalone in-place average of a small fp32 buffer (n <= max_elems), one
// workgroup, graph-capturable (seq lives in device memory).
hipError_t xgmi_allreduce_avg(const XgmiArgs& x, float* data, int n, hipStream_t s);

}  // namespace ptdt
