// Register-resident single-wave DDP step engine for Linear(Din, Dout) models.
//
// The flagship workload (ddp_gpus_torchrun.py:19-40 / SURVEY M4-M5: Linear(20,1),
// soft-target cross-entropy, SGD, 32 samples per rank per step, one all-reduce
// per step) is ~2k FLOPs per step: pure latency. The workgroup engine
// (fused_mlp.hip) keeps everything in LDS but still pays a chain of
// LDS round trips and s_barriers per phase. This engine removes both:
//
//   * ONE wave trains. Lane (j, p) owns row group j (j < 64 / L) and feature
//     chunk p (KP consecutive features, L = lanes per row); the group holds R
//     batch rows (row j + rho * 64/L), so the batch, the weights, the momentum
//     and the gradients all live in VGPRs.
//   * forward  : R*KP FMAs + a DPP row-group sum over the L lanes of a row;
//   * loss     : with R > 1 each of the first R lanes of a group computes one
//     row's loss and DPP broadcasts dL/dz to the group; with R == 1 the L
//     lanes of a row compute it redundantly (no exchange);
//   * backward : sum over the lane's R rows of g * x, then a rotation/permlane
//     column sum over the row groups -- every lane ends with the full-batch
//     gradient of ITS chunk, with the same bits in every lane (each butterfly
//     stage adds a+b / b+a). Cross-DPP-row permlane swaps cost ~4x a DPP add
//     (tools/microbench_isa.hip), so R > 1 trades them for local FMAs;
//   * all-reduce (world > 1): lanes of row q push the chunk to peer q and poll
//     peer q's contribution (xGMI one-shot, LL words, csrc/comm/xgmi.h), then
//     the same column sum adds the ranks -- identical on every rank;
//   * SGD      : each lane updates its own chunk in registers.
//   No s_barrier, no LDS traffic on the critical path. Batches are gathered
//   from the device-resident dataset NB steps ahead into register buffers
//   (indices read one step earlier still), so the L2 latency is hidden.
//   Waves 1-3 build the next epoch's sampler index list (Feistel permutation,
//   sampler.h) in LDS while wave 0 trains; the two meet at one s_barrier per
//   epoch.
// Configurations: L, R, KP (features per lane, zero padded), DOUT, the loss and
// whether an all-reduce exists are template parameters; anything else runs the
// workgroup engine.
#pragma once
#include <type_traits>
#include "common.h"
#include "kernels.h"
#include "sampler.h"

namespace ptdt {
namespace lw {

constexpr int kNB = kWavePrefetch;  // batches in flight (register buffers)
constexpr int kThreads = 256;    // wave 0 trains, waves 1-3 build index lists

__device__ __forceinline__ float swap16_add(float v) {
#pragma clang fp contract(off)
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(p[0]) + __int_as_float(p[1]);
}
__device__ __forceinline__ float swap32_add(float v) {
#pragma clang fp contract(off)
  auto p = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(p[0]) + __int_as_float(p[1]);
}

// Sum over the aligned group of L lanes of one batch row (L a power of two).
// L is a template parameter: a runtime L turns every stage into a branch.
// No FMA contraction inside the reductions: fma(g_i, x_i, g_j*x_j) on lane i and
// fma(g_j, x_j, g_i*x_i) on lane j round differently, and replicas would drift.
template <int L>
__device__ __forceinline__ float row_sum(float v) {
#pragma clang fp contract(off)
  if constexpr (L >= 2) v += dpp_f<kDppXor1>(v);
  if constexpr (L >= 4) v += dpp_f<kDppXor2>(v);
  if constexpr (L >= 8) v += dpp_f<kDppHalfMirror>(v);
  if constexpr (L >= 16) v += dpp_f<kDppMirror>(v);
  if constexpr (L >= 32) v = swap16_add(v);
  if constexpr (L >= 64) v = swap32_add(v);
  return v;
}

// Sum over all lanes with the same (lane % L): one feature chunk across rows.
// Rotations by 8,4,2,1 inside a 16-lane DPP row (row_ror), then the two
// permlane swaps. Each stage pairs lanes symmetrically, so every lane gets the
// same bits.
constexpr int kDppRor8 = 0x128, kDppRor4 = 0x124, kDppRor2 = 0x122, kDppRor1 = 0x121;
template <int L>
__device__ __forceinline__ float col_sum(float v) {
#pragma clang fp contract(off)
  if constexpr (L <= 8) v += dpp_f<kDppRor8>(v);
  if constexpr (L <= 4) v += dpp_f<kDppRor4>(v);
  if constexpr (L <= 2) v += dpp_f<kDppRor2>(v);
  if constexpr (L <= 1) v += dpp_f<kDppRor1>(v);
  if constexpr (L <= 16) v = swap16_add(v);
  if constexpr (L <= 32) v = swap32_add(v);
  return v;
}

// Optional per-phase s_memtime accounting (PersistArgs::stamps). Accumulators
// live in LDS, not SGPRs: the untimed build of the loop must not pay register
// pressure for diagnostics.
// Per-phase timers are compiled in only with -DPTDT_WAVE_STAMPS=1 (diagnostic
// builds): in the production build a tick is nothing, not even a branch --
// each skipped tick cost a taken branch plus an lgkmcnt(0) join per step.
#ifndef PTDT_WAVE_STAMPS
#define PTDT_WAVE_STAMPS 0
#endif
struct Ticks {
  bool on = false;
  int64_t prev = 0;
  unsigned long long* acc = nullptr;  // LDS [8]
  __device__ __forceinline__ void start() {
    if (PTDT_WAVE_STAMPS && on) prev = (int64_t)__builtin_amdgcn_s_memtime();
  }
  __device__ __forceinline__ void tick(int k) {
    if (PTDT_WAVE_STAMPS && on) {
      const int64_t t = (int64_t)__builtin_amdgcn_s_memtime();
      if (threadIdx.x == 0) acc[k] += (unsigned long long)(t - prev);
      prev = t;
    }
  }
};

// A/B switches of the chunked exchange's poll loop (tools/build_variant.py): PTDT_LL_PIPE = 1 keeps two
// poll rounds in flight; PTDT_LL_SLEEP = the s_sleep between single rounds (0: none). Shared-GPU
// rehearsal, 2,000 steps (profiles/r6_wave_exchange_poll_ab.jsonl): no sleep 1.56-1.57 / 1.78 us per
// step at W = 4 / 8, s_sleep 1 1.56-1.59 / 1.81-1.83, two rounds in flight 1.62 / 1.91-1.97.
#ifndef PTDT_LL_PIPE
#define PTDT_LL_PIPE 0
#endif
#ifndef PTDT_LL_SLEEP
#define PTDT_LL_SLEEP 0
#endif
// One-shot LL exchange of one lane's gradient chunk (csrc/comm/xgmi.h protocol):
// push the chunk to rank `peer` (when `active`), then poll rank `peer`'s chunk in
// this rank's buffer. Chunk elements: c*Din + k0 + k (k < KP, real when
// k0 + k < Din) and the biases nW + c. Every poll load is unconditional (padded
// slots re-read a real slot and are zeroed afterwards): loads under per-slot exec
// masks were issued one round trip at a time. Returns false after a poll timeout.
template <int KP, int DOUT>
__device__ __forceinline__ bool ll_exchange(bool active, uint64_t PTDT_GLOBAL* push_base,
                                            uint64_t PTDT_GLOBAL* poll_base, int my_rank, int peer, int world,
                                            int max_elems, uint32_t seq, int k0, int Din, bool hb, bool bias_lane,
                                            bool padded, const float (&gW)[DOUT][KP], const float (&gb)[DOUT],
                                            float (&v)[DOUT][KP], float (&vb)[DOUT], int* err, uint32_t max_polls,
                                            bool drop) {
  const int parity = (int)(seq & 1u);
  const int nW = DOUT * Din;
  const uint64_t hi = (uint64_t)seq << 32;
  if (!active) return true;
  uint64_t PTDT_GLOBAL* const dst = push_base + (int64_t)(parity * world + my_rank) * max_elems;
  uint64_t PTDT_GLOBAL* const src = poll_base + (int64_t)(parity * world + peer) * max_elems;
  if (drop) {  // fault injection: this rank's contribution never reaches its peers
  } else if (!padded) {
#pragma unroll
    for (int c = 0; c < DOUT; ++c)
#pragma unroll
      for (int k = 0; k < KP; ++k)
        __hip_atomic_store(dst + c * Din + k0 + k, hi | __float_as_uint(gW[c][k]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
#pragma unroll
    for (int c = 0; c < DOUT; ++c)
#pragma unroll
      for (int k = 0; k < KP; ++k)
        if (k0 + k < Din)
          __hip_atomic_store(dst + c * Din + k0 + k, hi | __float_as_uint(gW[c][k]), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (hb && bias_lane && !drop)
#pragma unroll
    for (int c = 0; c < DOUT; ++c)
      __hip_atomic_store(dst + nW + c, hi | __float_as_uint(gb[c]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#if PTDT_LL_PIPE
  // two poll rounds in flight (A/B variant): a round is re-issued as soon as it was checked, so a word
  // landing just after one round read the memory is caught by the other one
  uint64_t wa[DOUT][KP + 1], wb[DOUT][KP + 1];
  auto issue = [&](uint64_t (&w)[DOUT][KP + 1]) {
#pragma unroll
    for (int c = 0; c < DOUT; ++c) {
#pragma unroll
      for (int k = 0; k < KP; ++k)
        w[c][k] = __hip_atomic_load(src + c * Din + min(k0 + k, Din - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      w[c][KP] = __hip_atomic_load(src + (hb ? nW + c : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  };
  auto arrived = [&](const uint64_t (&w)[DOUT][KP + 1]) {
    bool all = true;
#pragma unroll
    for (int c = 0; c < DOUT; ++c)
#pragma unroll
      for (int k = 0; k <= KP; ++k) all &= (uint32_t)(w[c][k] >> 32) == seq;
    return all;
  };
  auto take = [&](const uint64_t (&w)[DOUT][KP + 1]) {
#pragma unroll
    for (int c = 0; c < DOUT; ++c) {
#pragma unroll
      for (int k = 0; k < KP; ++k) v[c][k] = k0 + k < Din ? __uint_as_float((uint32_t)w[c][k]) : 0.f;
      vb[c] = hb ? __uint_as_float((uint32_t)w[c][KP]) : 0.f;
    }
  };
  issue(wa);
  issue(wb);
  for (uint32_t polls = 0;; ++polls) {
    if (arrived(wa)) {
      take(wa);
      return true;
    }
    issue(wa);
    if (arrived(wb)) {
      take(wb);
      return true;
    }
    issue(wb);
    if (polls >= max_polls) {  // a peer is gone: fail loudly, never hang
      __hip_atomic_store((int PTDT_GLOBAL*)err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
  }
#else
  for (uint32_t polls = 0;; ++polls) {
    bool all = true;
#pragma unroll
    for (int c = 0; c < DOUT; ++c) {
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        const int e = c * Din + min(k0 + k, Din - 1);
        const uint64_t w = __hip_atomic_load(src + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        all &= (uint32_t)(w >> 32) == seq;
        v[c][k] = k0 + k < Din ? __uint_as_float((uint32_t)w) : 0.f;
      }
      // no bias: re-read element 0 (a real slot of this exchange) instead of branching
      const uint64_t w = __hip_atomic_load(src + (hb ? nW + c : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      all &= (uint32_t)(w >> 32) == seq;
      vb[c] = hb ? __uint_as_float((uint32_t)w) : 0.f;
    }
    if (all) return true;
    if (polls >= max_polls) {  // a peer is gone: fail loudly, never hang
      __hip_atomic_store((int PTDT_GLOBAL*)err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
#if PTDT_LL_SLEEP
    __builtin_amdgcn_s_sleep(PTDT_LL_SLEEP);
#endif
  }
#endif
}

// Uniform LL exchange for layout F (row slot i <-> rank i, csrc/comm/xgmi.h words) -- an
// alternative kept for tools/exchange_bench.hip, NOT used by the engines: measured on MI355X
// (profiles/r3_exchange_bench.jsonl) it is no faster than ll_exchange; the exchange is bound by
// the store-to-visible latency, not by the poll loop. Differences from ll_exchange:
//   * every lane polls a real slot: slot i < world (i != rank) polls rank i's chunk;
//     this rank's own slot and the slots >= world poll a peer's chunk too and then
//     take the own registers / 0. The poll loop is ONE uniform loop with a ballot
//     exit: no per-slot exec-mask branches, no divergent re-poll bookkeeping;
//   * two poll batches in flight: a batch is re-issued as soon as it was checked, so
//     a word landing just after one batch passed the memory is caught by the other;
//   * no s_sleep between polls (the wave has nothing else to issue).
// The values land exactly where ll_exchange puts them (v: rank i's chunk in slot i,
// own registers in slot `rank`, 0 above world), so the caller's row16_sum gives the
// same bits as before, on every rank. Returns false after a poll timeout (sets *err).
template <int KP, int DOUT>
__device__ __forceinline__ void ll_push_chunk(uint64_t PTDT_GLOBAL* push_base, int my_rank, int world, int max_elems,
                                              uint32_t seq, int k0, int Din, bool hb, bool bias_lane, bool padded,
                                              const float (&gW)[DOUT][KP], const float (&gb)[DOUT]) {
  const int parity = (int)(seq & 1u);
  const int nW = DOUT * Din;
  const uint64_t hi = (uint64_t)seq << 32;
  uint64_t PTDT_GLOBAL* const dst = push_base + (int64_t)(parity * world + my_rank) * max_elems;
  if (!padded) {
#pragma unroll
    for (int c = 0; c < DOUT; ++c)
#pragma unroll
      for (int k = 0; k < KP; ++k)
        __hip_atomic_store(dst + c * Din + k0 + k, hi | __float_as_uint(gW[c][k]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
#pragma unroll
    for (int c = 0; c < DOUT; ++c)
#pragma unroll
      for (int k = 0; k < KP; ++k)
        if (k0 + k < Din)
          __hip_atomic_store(dst + c * Din + k0 + k, hi | __float_as_uint(gW[c][k]), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (hb && bias_lane)
#pragma unroll
    for (int c = 0; c < DOUT; ++c)
      __hip_atomic_store(dst + nW + c, hi | __float_as_uint(gb[c]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Poll half of ll_exchange_u: slot `slot` < world polls rank `slot`'s chunk (every rank's,
// own included when `own_from_memory`, i.e. the own chunk was self-pushed); other slots poll
// a real peer's chunk and take 0 (or the own registers for slot == rank without self-push).
template <int KP, int DOUT>
__device__ __forceinline__ bool ll_poll_chunk(uint64_t PTDT_GLOBAL* poll_base, int my_rank, int slot, int world,
                                              int max_elems, uint32_t seq, int k0, int Din, bool hb,
                                              bool own_from_memory, const float (&gW)[DOUT][KP],
                                              const float (&gb)[DOUT], float (&v)[DOUT][KP], float (&vb)[DOUT],
                                              int* err, uint32_t max_polls) {
  constexpr int NS = DOUT * (KP + 1);
  const int parity = (int)(seq & 1u);
  const int nW = DOUT * Din;
  const bool mem = slot < world && (slot != my_rank || own_from_memory);
  const int src_rank = mem ? slot : (my_rank + 1 == world ? 0 : my_rank + 1);  // some real chunk
  uint64_t PTDT_GLOBAL* const src = poll_base + (int64_t)(parity * world + src_rank) * max_elems;
  int off[NS];
#pragma unroll
  for (int c = 0; c < DOUT; ++c) {
#pragma unroll
    for (int k = 0; k < KP; ++k) off[c * (KP + 1) + k] = c * Din + min(k0 + k, Din - 1);
    off[c * (KP + 1) + KP] = hb ? nW + c : 0;  // no bias: re-read a real slot of this exchange
  }
  uint64_t wa[NS], wb[NS];
  auto issue = [&](uint64_t (&w)[NS]) {
#pragma unroll
    for (int s = 0; s < NS; ++s) w[s] = __hip_atomic_load(src + off[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  };
  auto missing = [&](const uint64_t (&w)[NS]) {
    bool m = false;
#pragma unroll
    for (int s = 0; s < NS; ++s) m |= (uint32_t)(w[s] >> 32) != seq;
    return __builtin_amdgcn_ballot_w64(m) != 0;  // uniform
  };
  const bool own = slot == my_rank && !own_from_memory;
  auto take = [&](const uint64_t (&w)[NS]) {
#pragma unroll
    for (int c = 0; c < DOUT; ++c) {
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        const float x = __uint_as_float((uint32_t)w[c * (KP + 1) + k]);
        v[c][k] = own ? gW[c][k] : ((mem && k0 + k < Din) ? x : 0.f);
      }
      const float xb = __uint_as_float((uint32_t)w[c * (KP + 1) + KP]);
      vb[c] = own ? gb[c] : ((mem && hb) ? xb : 0.f);
    }
  };
  issue(wa);
  issue(wb);
  for (uint32_t polls = 0;; ++polls) {
    if (!missing(wa)) {
      take(wa);
      return true;
    }
    issue(wa);
    if (!missing(wb)) {
      take(wb);
      return true;
    }
    issue(wb);
    if (polls >= max_polls) {  // a peer is gone: fail loudly, never hang
      __hip_atomic_store((int PTDT_GLOBAL*)err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      take(wa);
      return false;
    }
  }
}

template <int KP, int DOUT>
__device__ __forceinline__ bool ll_exchange_u(bool push, uint64_t PTDT_GLOBAL* push_base,
                                              uint64_t PTDT_GLOBAL* poll_base, int my_rank, int slot, int world,
                                              int max_elems, uint32_t seq, int k0, int Din, bool hb, bool bias_lane,
                                              bool padded, const float (&gW)[DOUT][KP], const float (&gb)[DOUT],
                                              float (&v)[DOUT][KP], float (&vb)[DOUT], int* err,
                                              uint32_t max_polls) {
  if (push) ll_push_chunk<KP, DOUT>(push_base, my_rank, world, max_elems, seq, k0, Din, hb, bias_lane, padded, gW, gb);
  return ll_poll_chunk<KP, DOUT>(poll_base, my_rank, slot, world, max_elems, seq, k0, Din, hb, false, gW, gb, v, vb,
                                 err, max_polls);
}

// Packed LL exchange for layout F (tools/exchange_bench.hip variant 6): the rank's npw
// values (DOUT*Din weights + the biases) are staged in LDS and travel as npw CONSECUTIVE
// words per peer -- lane f of the NT store / poll instructions handles (peer f / npw, word
// f % npw), so every peer's words go out in ~2 cache lines and all peers' stores and polls
// are in flight together. ll_exchange instead stores each lane's KP-value chunk to its row
// slot's peer (6 store instructions hitting the same 1-2 lines per peer for Linear(20,1)):
// uncached stores cost per transaction, and the exchange measured ~30 % longer at W = 2 and
// ~2x at W = 8 (profiles/r3_exchange_bench.jsonl). After the polls, every lane sums ITS
// chunk's words over the ranks in rank order from LDS: the same bits on every rank, and
// the same order as the standalone xgmi_allreduce_avg kernel.
// PackPlan: per-lane (peer, word) of the NT instructions, computed once per launch.
template <int NT>
struct PackPlan {
  int pr[NT], wd[NT];  // peer rank (-1: idle lane), word index
};
template <int NT>
__device__ __forceinline__ PackPlan<NT> pack_plan(int npw, int world, int my_rank, int lane) {
  PackPlan<NT> pp;
  const int nf = npw * (world - 1);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int f = lane + 64 * t;
    const int pi = f / npw;
    pp.wd[t] = f - pi * npw;
    pp.pr[t] = f < nf ? (pi < my_rank ? pi : pi + 1) : -1;
  }
  return pp;
}
// stg: LDS [npw] (own values, written by the caller), pol: LDS [world][npw]. Returns false
// after a poll timeout (sets *err). drop: fault injection -- pushes to the peers are skipped.
template <int NT>
__device__ __forceinline__ bool ll_exchange_packed(const PackPlan<NT>& pp, const XgmiArgs& x, uint32_t seq, int npw,
                                                   const float* stg, float* pol, int lane, bool drop) {
  const int parity = (int)(seq & 1u);
  const uint64_t hi = (uint64_t)seq << 32;
  if (!drop) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (pp.pr[t] < 0) continue;
      uint64_t PTDT_GLOBAL* base = nullptr;  // peers[] selected with uniform compares (no scratch copy)
#pragma unroll
      for (int r = 0; r < kXgmiMaxRanks; ++r)
        if (pp.pr[t] == r) base = (uint64_t PTDT_GLOBAL*)x.peers[r];
      __hip_atomic_store(base + (int64_t)(parity * x.world + x.rank) * x.max_elems + pp.wd[t],
                         hi | __float_as_uint(stg[pp.wd[t]]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  const uint64_t PTDT_GLOBAL* const local = (const uint64_t PTDT_GLOBAL*)x.local;
  const int alt = x.rank + 1 == x.world ? 0 : x.rank + 1;  // idle lanes re-read a real slot
  uint64_t w[NT];
  auto issue = [&]() {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const bool on = pp.pr[t] >= 0;
      w[t] = __hip_atomic_load(local + (int64_t)(parity * x.world + (on ? pp.pr[t] : alt)) * x.max_elems +
                                   (on ? pp.wd[t] : 0),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  };
  issue();
  bool ok = true;
  for (uint32_t polls = 0;; ++polls) {
    bool m = false;
#pragma unroll
    for (int t = 0; t < NT; ++t) m |= pp.pr[t] >= 0 && (uint32_t)(w[t] >> 32) != seq;
    if (__builtin_amdgcn_ballot_w64(m) == 0) break;
    if (polls >= x.max_polls) {  // a peer is gone: fail loudly, never hang
      __hip_atomic_store((int PTDT_GLOBAL*)x.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      ok = false;
      break;
    }
    issue();
  }
#pragma unroll
  for (int t = 0; t < NT; ++t)
    if (pp.pr[t] >= 0) pol[pp.pr[t] * npw + pp.wd[t]] = __uint_as_float((uint32_t)w[t]);
  for (int f = lane; f < npw; f += 64) pol[x.rank * npw + f] = stg[f];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its LDS ops complete in order
  return ok;
}

// Pair exchange of layout F at world 2 (tools/exchange_bench.hip variant 4): the rank's npw <= 64
// values (DOUT*Din weights, then the biases) are staged in LDS and travel as npw consecutive LL
// words in ONE store instruction to the peer, and come back with ONE poll instruction -- against
// the chunked exchange's per-row-slot stores and polls (W = 2 rehearsal: 1,799 vs 2,369 cycles,
// profiles/r3_allreduce.md). The two-term sum x0 + x1 is the chunked path's row sum over
// {x0, x1, 0, ...} (adding zeros is exact), so both ranks -- and both paths -- get the same values
// (up to the sign of an exact zero). xs: LDS [128] (staging, then the averages).
template <int KP, int DOUT>
__device__ __forceinline__ bool ll_exchange_pair(const XgmiArgs& x, uint32_t seq, int q, int i, int lane, int Din,
                                                 float (&gW)[DOUT][KP], float (&gb)[DOUT], float* xs, float inv_w,
                                                 bool drop) {
  const int k0 = q * KP, nW = DOUT * Din, npw = nW + DOUT;
  if (i == 0) {
#pragma unroll
    for (int c = 0; c < DOUT; ++c) {
#pragma unroll
      for (int k = 0; k < KP; ++k)
        if (k0 + k < Din) xs[c * Din + k0 + k] = gW[c][k];
      if (q == 0) xs[nW + c] = gb[c];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // one wave: its LDS ops complete in order
  const bool on = lane < npw;
  const float mine = on ? xs[lane] : 0.f;
  const int parity = (int)(seq & 1u), peer = 1 - x.rank;
  const uint64_t hi = (uint64_t)seq << 32;
  if (!drop && on) {
    uint64_t PTDT_GLOBAL* base = nullptr;  // uniform selects, no scratch copy of peers[]
#pragma unroll
    for (int r = 0; r < 2; ++r)
      if (peer == r) base = (uint64_t PTDT_GLOBAL*)x.peers[r];
    __hip_atomic_store(base + (int64_t)(parity * 2 + x.rank) * x.max_elems + lane, hi | __float_as_uint(mine),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const uint64_t PTDT_GLOBAL* const src =
      (const uint64_t PTDT_GLOBAL*)x.local + (int64_t)(parity * 2 + peer) * x.max_elems + (on ? lane : 0);
  uint64_t w = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  bool ok = true;
  for (uint32_t polls = 0; __builtin_amdgcn_ballot_w64(on && (uint32_t)(w >> 32) != seq) != 0; ++polls) {
    if (polls >= x.max_polls) {  // the peer is gone: fail loudly, never hang
      __hip_atomic_store((int PTDT_GLOBAL*)x.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      ok = false;
      break;
    }
    w = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const float other = __uint_as_float((uint32_t)w);
  xs[64 + lane] = (x.rank == 0 ? mine + other : other + mine) * inv_w;  // rank order
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int c = 0; c < DOUT; ++c) {
#pragma unroll
    for (int k = 0; k < KP; ++k) gW[c][k] = k0 + k < Din ? xs[64 + c * Din + k0 + k] : 0.f;
    gb[c] = xs[64 + nW + c];
  }
  return ok;
}

template <int R, int KP, int DOUT, int RY>
struct Batch {
  float x[R][KP];
  float y[RY][DOUT];
  int yi[RY];
  int nb;        // rows in this batch (last batch of an epoch may be short)
  float cg, cl;  // layout F: dL/dz scale (grad_scale / rows) and loss scale (1 / rows) of this batch
};

// quad_perm broadcast of lane `src` of each aligned group of L (2 or 4) lanes
template <int L, int SRC>
constexpr int bcast_ctrl() {
  return L == 4 ? SRC * 0x55 : (SRC | (SRC << 2) | ((2 + SRC) << 4) | ((2 + SRC) << 6));
}

template <int L, int R, int KP, int DOUT, int LOSS, bool AR>
__global__ void __launch_bounds__(kThreads) linear_wave_kernel(FusedMlpArgs a, PersistArgs pa) {
  // R > 1: the first R lanes of each group each compute one row's loss
  constexpr bool SPLIT = R > 1 && (L == 2 || L == 4) && R <= L;
  constexpr int RY = SPLIT ? 1 : R;  // target rows each lane loads
  constexpr int RG = 64 / L;         // row groups
  extern __shared__ int elist[];     // [2][estride] sampler index lists (epoch parity)
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int B = a.B, Din = a.Din;
  const int estride = al4(pa.num_samples);
  const int S = (pa.num_samples + B - 1) / B;  // steps per epoch
  const int e0 = pa.cursor[0], j0 = pa.cursor[1];
  const int64_t pos0 = (int64_t)e0 * S + j0;
  const int n = pa.n_steps;
  const int T = (int)((pos0 + n - 1) / S - pos0 / S);  // epoch transitions inside this launch
  auto list = [&](int e) { return elist + (e & 1) * estride; };

  // only the first epoch's list is on the path to step 0 (stale reads past the
  // launch are clamped below); e0+1 is built by the helpers after the barrier
  const ListCache lc{pa.lcache, pa.ltag, estride};
  rank_epoch_indices_or(given_list(pa, e0), list(e0), (uint32_t)pa.N, pa.W, pa.rank, pa.num_samples, pa.seed, e0, pa.shuffle,
                     (int)threadIdx.x, kThreads, lc);
  __syncthreads();
  if (wave != 0) {
    // producers: after the trainer starts prefetching epoch e0+i, the list of
    // e0+i-1 is dead; build e0+i+1 into its slot before the next transition.
    const int ht = (int)threadIdx.x - 64;
    if (ht == 0 && pa.idx == nullptr) list_cache_publish(lc, e0);
    if (T > 0)
      rank_epoch_indices_or(given_list(pa, e0 + 1), list(e0 + 1), (uint32_t)pa.N, pa.W, pa.rank, pa.num_samples, pa.seed, e0 + 1,
                            pa.shuffle, ht, kThreads - 64, lc);
    for (int i = 1; i <= T; ++i) {
      __syncthreads();
      if (ht == 0 && pa.idx == nullptr) list_cache_publish(lc, e0 + i);
      if (i < T)
        rank_epoch_indices_or(given_list(pa, e0 + i + 1), list(e0 + i + 1), (uint32_t)pa.N, pa.W, pa.rank, pa.num_samples, pa.seed, e0 + i + 1,
                           pa.shuffle, ht, kThreads - 64, lc);
    }
    return;
  }

  // ------------------------------------------------------------------ trainer wave
  const int lane = (int)threadIdx.x;
  const int j = lane / L, p = lane % L;    // row group, feature chunk
  const int k0 = p * KP;
  const int rho_y = SPLIT ? min(p, R - 1) : 0;  // the row whose loss this lane computes (SPLIT)
  const bool hb = a.has_bias != 0;
  const bool use_mom = a.mom != nullptr && a.momentum != 0.f;
  const float lr = a.lr, mu = a.momentum, damp = a.dampening, wd = a.weight_decay;
  const int nesterov = a.nesterov;
  const auto X = gptr(a.X);
  const int nW = DOUT * Din;

  float W[DOUT][KP], M[DOUT][KP], Wb[DOUT], Mb[DOUT];
  {
    const auto P = gptr(a.P);
#pragma unroll
    for (int c = 0; c < DOUT; ++c) {
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        const bool in = k0 + k < Din;
        W[c][k] = in ? P[c * Din + k0 + k] : 0.f;
        M[c][k] = (in && use_mom) ? gptr(a.mom)[c * Din + k0 + k] : 0.f;
      }
      Wb[c] = hb ? P[nW + c] : 0.f;
      Mb[c] = (hb && use_mom) ? gptr(a.mom)[nW + c] : 0.f;
    }
  }
  int opt_step = a.opt_step ? *a.opt_step : 0;
  const XgmiArgs& ar = a.ar;
  const int world = AR ? ar.world : 1;  // AR == false: single rank, no all-reduce code at all
  // this lane's push target (row group q pushes to rank q) and poll source,
  // selected once with uniform compares: indexing peers[] by a lane value would
  // spill the argument array to scratch
  uint64_t PTDT_GLOBAL* push_dst = nullptr;
#pragma unroll
  for (int q = 0; q < kXgmiMaxRanks; ++q)
    if (j == q && q < world) push_dst = (uint64_t PTDT_GLOBAL*)ar.peers[q];
  uint64_t PTDT_GLOBAL* const poll_src = (uint64_t PTDT_GLOBAL*)ar.local;
  const int my_rank = ar.rank, max_elems = ar.max_elems;
  float PTDT_GLOBAL* const losses = gptr_w(pa.losses);
  uint32_t seq = AR ? *ar.seq : 0u;
  bool failed = AR && *ar.err != 0;  // a peer already timed out earlier: do not wait again
  const float inv_w = 1.f / (float)world;

  // Feature slots past Din (L * KP > Din) read the zero padding of X (the host
  // guarantees ldx >= L * KP and zeros there): their gradient is 0, W stays 0.
  const int ldx = a.ldx > 0 ? a.ldx : Din;
  // index lookahead: the dataset rows of the next batch are read from LDS one
  // fetch before the gather that uses them
  int ie = e0, ij = j0, barriers = 0;
  int sel_next[R], sel_y_next = 0, nb_next = 0;
  // Always called (also for the kNB positions past this launch, whose lists may
  // be stale): no conditional loads in the loop, so the waitcnt pass can count
  // the outstanding prefetches exactly instead of falling back to vmcnt(0).
  const uint32_t N = (uint32_t)pa.N;
  auto read_index = [&]() {
    if (ij == 0 && ie != e0 && barriers < T) {  // new epoch: its list is ready, the old one free
      __syncthreads();
      ++barriers;
    }
    nb_next = min(B, pa.num_samples - ij * B);
#pragma unroll
    for (int rho = 0; rho < R; ++rho) {  // rows past the batch re-read its last row
      const int sel = list(ie)[ij * B + min(rho * RG + j, nb_next - 1)];
      sel_next[rho] = (uint32_t)sel < N ? sel : 0;
    }
    if constexpr (SPLIT) {  // own row's index read directly (selecting by a lane value spills)
      const int sel = list(ie)[ij * B + min(rho_y * RG + j, nb_next - 1)];
      sel_y_next = (uint32_t)sel < N ? sel : 0;
    }
    if (++ij == S) {
      ij = 0;
      ++ie;
    }
  };
  auto fetch = [&](Batch<R, KP, DOUT, RY>& f) {
    // Unconditional loads (no exec-mask branches), immediate offsets from one
    // address per row: rows past the batch re-read a valid row and get g = 0.
    f.nb = nb_next;
#pragma unroll
    for (int rho = 0; rho < R; ++rho) {
      const auto xr = X + (int64_t)sel_next[rho] * ldx + k0;
#pragma unroll
      for (int k = 0; k < KP; ++k) f.x[rho][k] = xr[k];
    }
#pragma unroll
    for (int ry = 0; ry < RY; ++ry) {
      const int sel = SPLIT ? sel_y_next : sel_next[ry];
      if constexpr (LOSS == kLossCEIndex) {
        f.yi[ry] = reinterpret_cast<const int*>(a.Yi)[2 * (int64_t)sel];  // low dword (see mlp_tp.hip)
      } else {
#pragma unroll
        for (int c = 0; c < DOUT; ++c) f.y[ry][c] = gptr(a.Yf)[(int64_t)sel * DOUT + c];
      }
    }
    read_index();
  };

  Ticks tk;
  tk.on = pa.stamps != nullptr;
  tk.acc = reinterpret_cast<unsigned long long*>(elist + 2 * estride);
  if (tk.on && lane == 0)
    for (int k = 0; k < 8; ++k) tk.acc[k] = 0ull;
  const float inv_full = 1.f / (float)((LOSS == kLossMSE) ? B * DOUT : B);
  const int64_t t_begin = tk.on ? (int64_t)__builtin_amdgcn_s_memtime() : 0;
  const int64_t r_begin = tk.on ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;

  // loss and dL/dz of one row: l (summed loss), cnt (CE index: 1 if counted)
  auto row_loss = [&](const float* z, const float* y, int yi, bool valid, float* g, float& l, float& cnt) {
    l = 0.f;
    cnt = 0.f;
    if constexpr (LOSS == kLossMSE) {
#pragma unroll
      for (int c = 0; c < DOUT; ++c) {
        const float df = z[c] - y[c];
        l = fmaf(df, df, l);
        g[c] = 2.f * df;
      }
    } else if constexpr (DOUT == 1) {
      // one class: log_softmax(z) = z - z (0, or NaN for a non-finite z) -- no exp/log
      const float ls0 = z[0] - z[0];
      if constexpr (LOSS == kLossCESoft) {
        l = -y[0] * ls0;
        g[0] = (ls0 + 1.f) * y[0] - y[0];
      } else {
        const bool use = yi != a.ignore_index;
        g[0] = use ? (ls0 + 1.f) - (yi == 0 ? 1.f : 0.f) : 0.f;
        l = use ? -(yi == 0 ? ls0 : 0.f) : 0.f;
        cnt = use ? 1.f : 0.f;
      }
    } else {
      float m = z[0];
#pragma unroll
      for (int c = 1; c < DOUT; ++c) m = fmaxf(m, z[c]);
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < DOUT; ++c) se += __expf(z[c] - m);
      // se >= 1 (the max term is exp(0)): the hardware log2 needs no denormal fix-up
      const float lse = m + __builtin_amdgcn_logf(se) * 0.6931471805599453f;
      if constexpr (LOSS == kLossCESoft) {
        float tsum = 0.f;
#pragma unroll
        for (int c = 0; c < DOUT; ++c) {
          tsum += y[c];
          l -= y[c] * (z[c] - lse);
        }
#pragma unroll
        for (int c = 0; c < DOUT; ++c) g[c] = __expf(z[c] - lse) * tsum - y[c];
      } else {
        const bool use = yi != a.ignore_index;
        float zy = 0.f;
#pragma unroll
        for (int c = 0; c < DOUT; ++c) {
          zy = c == yi ? z[c] : zy;
          g[c] = use ? __expf(z[c] - lse) - (c == yi ? 1.f : 0.f) : 0.f;
        }
        l = use ? lse - zy : 0.f;
        cnt = use ? 1.f : 0.f;
      }
    }
    if (!valid) {
#pragma unroll
      for (int c = 0; c < DOUT; ++c) g[c] = 0.f;
      l = 0.f;
      cnt = 0.f;
    }
  };

  auto train = [&](Batch<R, KP, DOUT, RY>& f, int step) {
    const int nb = f.nb;
    // ---- forward
    float z[R][DOUT];
#pragma unroll
    for (int rho = 0; rho < R; ++rho) {
#pragma unroll
      for (int c = 0; c < DOUT; ++c) {
        float acc0 = 0.f, acc1 = 0.f;
#pragma unroll
        for (int k = 0; k < KP; k += 2) {
          acc0 = fmaf(f.x[rho][k], W[c][k], acc0);
          if (k + 1 < KP) acc1 = fmaf(f.x[rho][k + 1], W[c][k + 1], acc1);
        }
        z[rho][c] = row_sum<L>(acc0 + acc1) + Wb[c];
      }
    }
    tk.tick(1);
    // ---- loss and dL/dz
    float g[R][DOUT], lsum = 0.f, csum = 0.f;
    if constexpr (SPLIT) {
      float zs[DOUT];
#pragma unroll
      for (int c = 0; c < DOUT; ++c) {
        zs[c] = z[0][c];
#pragma unroll
        for (int rho = 1; rho < R; ++rho) zs[c] = rho_y == rho ? z[rho][c] : zs[c];
      }
      float gs[DOUT], l, cnt;
      row_loss(zs, f.y[0], f.yi[0], rho_y * RG + j < nb, gs, l, cnt);
      const bool owner = p < R;  // lanes p >= R duplicated row R-1: not counted
      lsum = owner ? l : 0.f;
      csum = owner ? cnt : 0.f;
#pragma unroll
      for (int c = 0; c < DOUT; ++c) {
        g[0][c] = dpp_f<bcast_ctrl<L, 0>()>(gs[c]);
        if constexpr (R > 1) g[1][c] = dpp_f<bcast_ctrl<L, 1>()>(gs[c]);
        if constexpr (R > 2) g[2][c] = dpp_f<bcast_ctrl<L, 2>()>(gs[c]);
        if constexpr (R > 3) g[3][c] = dpp_f<bcast_ctrl<L, 3>()>(gs[c]);
      }
    } else {
#pragma unroll
      for (int rho = 0; rho < R; ++rho) {
        float l, cnt;
        row_loss(z[rho], f.y[rho], f.yi[rho], rho * RG + j < nb, g[rho], l, cnt);
        lsum += l;
        csum += cnt;
      }
      if (p != 0) {  // the L lanes of a row computed the same loss: count it once
        lsum = 0.f;
        csum = 0.f;
      }
    }
    float inv_denom;
    if constexpr (LOSS == kLossCEIndex) {
      csum = wave_sum(csum);  // the one data-dependent denominator
      inv_denom = 1.f / (csum > 0.f ? csum : 1.f);
    } else {  // division only for a short last batch
      inv_denom = nb == B ? inv_full : 1.f / (float)((LOSS == kLossMSE) ? nb * DOUT : nb);
    }
    const float coef = a.grad_scale * inv_denom;
    tk.tick(2);
    // ---- backward: full-batch gradient of this lane's chunk, in every lane
    float gW[DOUT][KP], gb[DOUT];
#pragma unroll
    for (int c = 0; c < DOUT; ++c) {
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        float t = g[0][c] * f.x[0][k];
#pragma unroll
        for (int rho = 1; rho < R; ++rho) t = fmaf(g[rho][c], f.x[rho][k], t);
        gW[c][k] = col_sum<L>(t) * coef;
      }
      float tb = g[0][c];
#pragma unroll
      for (int rho = 1; rho < R; ++rho) tb += g[rho][c];
      gb[c] = col_sum<L>(tb) * coef;
    }
    tk.tick(3);
    // ---- all-reduce over ranks (average): row group q <-> rank q
    if (AR && !failed) {
      seq += 1u;
      float v[DOUT][KP], vb[DOUT];
#pragma unroll
      for (int c = 0; c < DOUT; ++c) {  // own contribution from registers, rows >= world add 0
        vb[c] = j == my_rank ? gb[c] : 0.f;
#pragma unroll
        for (int k = 0; k < KP; ++k) v[c][k] = j == my_rank ? gW[c][k] : 0.f;
      }
      const bool ok = ll_exchange<KP, DOUT>(j < world && j != my_rank, push_dst, poll_src, my_rank, j, world,
                                            max_elems, seq, k0, Din, hb, p == 0, L * KP != Din, gW, gb, v, vb,
                                            ar.err, ar.max_polls, ar.drop_push != 0u && seq >= ar.drop_push);
      failed = !ok;
      failed = __any(failed);
#pragma unroll
      for (int c = 0; c < DOUT; ++c) {
#pragma unroll
        for (int k = 0; k < KP; ++k) gW[c][k] = col_sum<L>(v[c][k]) * inv_w;
        gb[c] = col_sum<L>(vb[c]) * inv_w;
      }
    }
    tk.tick(4);
    // ---- SGD (torch.optim.SGD semantics) on this lane's chunk; unswitched on
    // momentum so the unrolled body has no per-element branches
    const bool first = opt_step == 0;
    auto sgd_all = [&](auto mom_tag) {
      constexpr bool MOM = decltype(mom_tag)::value;
      auto upd = [&](float& w, float& m, float gr) {
        float d = fmaf(wd, w, gr);
        if constexpr (MOM) {
          const float buf = first ? d : fmaf(mu, m, (1.f - damp) * d);
          m = buf;
          d = nesterov ? fmaf(mu, buf, d) : buf;
        }
        w = fmaf(-lr, d, w);
      };
#pragma unroll
      for (int c = 0; c < DOUT; ++c) {
#pragma unroll
        for (int k = 0; k < KP; ++k) upd(W[c][k], M[c][k], gW[c][k]);
        upd(Wb[c], Mb[c], gb[c]);
        Wb[c] = hb ? Wb[c] : 0.f;  // no bias: stays 0 (select, not a branch)
      }
    };
    if (use_mom) sgd_all(std::true_type{});
    else sgd_all(std::false_type{});
    ++opt_step;
    if (step == n - 1 && j == 0) {  // the DDP bucket keeps the last step's averaged gradients
      const auto Gw = gptr_w(a.G);
#pragma unroll
      for (int c = 0; c < DOUT; ++c) {
#pragma unroll
        for (int k = 0; k < KP; ++k)
          if (k0 + k < Din) Gw[c * Din + k0 + k] = gW[c][k];
        if (hb && p == 0) Gw[nW + c] = gb[c];
      }
    }
    // ---- loss report (off the critical path: nothing waits on it); every lane
    // stores the same value to the same address: no exec-mask branch
    const float ls = wave_sum(lsum);
    if constexpr (LOSS == kLossCEIndex) losses[step] = csum > 0.f ? ls * inv_denom : NAN;
    else losses[step] = ls * inv_denom;
    tk.tick(5);
  };

  Batch<R, KP, DOUT, RY> buf[kNB];
  tk.start();
  read_index();
#pragma unroll
  for (int u = 0; u < kNB; ++u) fetch(buf[u]);
  tk.tick(0);
  // main loop: whole groups of kNB steps, straight-line body (every fetch
  // unconditional); then the < kNB tail steps
  int done = 0;
  const int nfull = n - n % kNB;
  while (done < nfull && !failed) {
#pragma unroll
    for (int u = 0; u < kNB; ++u) {
      train(buf[u], done + u);
      fetch(buf[u]);
      tk.tick(0);
    }
    done += kNB;
  }
#pragma unroll
  for (int u = 0; u < kNB - 1; ++u) {
    if (done < n && !failed) {
      train(buf[u], done);
      ++done;
    }
  }
  // a failed all-reduce stops training early: still meet the producers at every barrier
  while (barriers < T) {
    __syncthreads();
    ++barriers;
  }

  // ---- write back resident state (lanes of row group 0 hold every chunk)
  if (j == 0) {
    const auto Pw = gptr_w(a.P);
#pragma unroll
    for (int c = 0; c < DOUT; ++c) {
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        if (k0 + k < Din) {
          Pw[c * Din + k0 + k] = W[c][k];
          if (use_mom) a.mom[c * Din + k0 + k] = M[c][k];
        }
      }
      if (hb && p == 0) {
        Pw[nW + c] = Wb[c];
        if (use_mom) a.mom[nW + c] = Mb[c];
      }
    }
  }
  if (lane == 0) {
    const int64_t pos = pos0 + done;
    pa.cursor[0] = (int)(pos / S);
    pa.cursor[1] = (int)(pos % S);
    if (a.opt_step) *a.opt_step = opt_step;
    if (AR) *ar.seq = seq;
    if (tk.on) {
      // [0] fetch (index read + gather issue + epoch barrier), [1] forward, [2] loss,
      // [3] backward, [4] all-reduce, [5] sgd + loss report
      for (int k = 0; k < 6; ++k) pa.stamps[k] += (int64_t)tk.acc[k];
      pa.stamps[7] += (int64_t)__builtin_amdgcn_s_memtime() - t_begin;
      pa.stamps[8] += (int64_t)__builtin_amdgcn_s_memrealtime() - r_begin;
    }
  }
}

// ============================================================================
// Layout F ("features across DPP rows"): lane (q, i) = (lane / 16, lane % 16).
// DPP row q owns feature group q (KP consecutive features, 4 * KP >= Din);
// row slot i holds batch rows i + 16 * rho, rho < R (B <= 16 R).
//   forward : the 4 feature-group partial logits of a row meet with permlane
//             swaps; with DOUT == 1 the R rows are reduce-scattered in pairs
//             (one swap per pair and stage, no register copies), so each lane
//             ends with ONE row's logit and computes that row's loss;
//   dL/dz   : all-gathered back with the same swaps;
//   backward: the column sum over the 16 row slots of a DPP row is 4 row_ror
//             DPP adds -- no permlane at all (vs 2 per gradient element when
//             rows span DPP rows). Measured issue costs (tools/microbench_isa):
//             DPP add ~5.6 cycles, permlane swap ~20.
// All reductions pair lanes symmetrically (a+b / b+a): every lane that holds
// a value holds the same bits.

struct F2 {
  float a, b;
};
// permlane16_swap(A, B): A' = rows [A0, B0, A2, B2], B' = rows [A1, B1, A3, B3]
__device__ __forceinline__ F2 pl16(float a, float b) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_int(a), __float_as_int(b), false, false);
  return {__int_as_float(p[0]), __int_as_float(p[1])};
}
// permlane32_swap(A, B): A' = rows [A0, A1, B0, B1], B' = rows [A2, A3, B2, B3]
__device__ __forceinline__ F2 pl32(float a, float b) {
  auto p = __builtin_amdgcn_permlane32_swap(__float_as_int(a), __float_as_int(b), false, false);
  return {__int_as_float(p[0]), __int_as_float(p[1])};
}
// stage-16 reduce-scatter of a pair: rows [a0+a1, b0+b1, a2+a3, b2+b3]
__device__ __forceinline__ float rs16(float a, float b) {
#pragma clang fp contract(off)
  const F2 r = pl16(a, b);
  return r.a + r.b;
}
// stage-32 reduce-scatter of a pair: rows [a0+a2, a1+a3, b0+b2, b1+b3]
__device__ __forceinline__ float rs32(float a, float b) {
#pragma clang fp contract(off)
  const F2 r = pl32(a, b);
  return r.a + r.b;
}
// full sum over the 4 DPP rows, in every lane
__device__ __forceinline__ float allrows(float v) {
  const float s = rs16(v, v);
  return rs32(s, s);
}
// sum over the 16 lanes of a DPP row (row_ror 8, 4, 2, 1), in every lane of the row
__device__ __forceinline__ float row16_sum(float v) {
#pragma clang fp contract(off)
  v += dpp_f<kDppRor8>(v);
  v += dpp_f<kDppRor4>(v);
  v += dpp_f<kDppRor2>(v);
  v += dpp_f<kDppRor1>(v);
  return v;
}
// row16_sum of N values at once. For N == 6 (KP = 5 features + the bias: the flagship Linear(20,1)
// chunk) the 24 DPP adds are ONE asm block, stage-major, so each value's next stage is 6 instructions
// after its previous one (no s_nop: DPP reads a VGPR 2 wait states after its VALU write) and every
// stage is a single v_add_f32_dpp. Left to the compiler, the chains were either finished one after
// the other with an s_nop between every two stages, or their last add sank past the step's
// epoch-barrier branch and was no longer fused with its DPP move (v_mov + v_mov_dpp + v_add per value).
// The sums are the same bits as row16_sum (v + ror(v), same stage order).
template <int N>
__device__ __forceinline__ void row16_sum_n(float* v) {
  if constexpr (N == 6) {
#define PTDT_R16(ROR)                                                         \
  "v_add_f32_dpp %0, %0, %0 row_ror:" #ROR " row_mask:0xf bank_mask:0xf\n\t" \
  "v_add_f32_dpp %1, %1, %1 row_ror:" #ROR " row_mask:0xf bank_mask:0xf\n\t" \
  "v_add_f32_dpp %2, %2, %2 row_ror:" #ROR " row_mask:0xf bank_mask:0xf\n\t" \
  "v_add_f32_dpp %3, %3, %3 row_ror:" #ROR " row_mask:0xf bank_mask:0xf\n\t" \
  "v_add_f32_dpp %4, %4, %4 row_ror:" #ROR " row_mask:0xf bank_mask:0xf\n\t" \
  "v_add_f32_dpp %5, %5, %5 row_ror:" #ROR " row_mask:0xf bank_mask:0xf\n\t"
    asm volatile("s_nop 1\n\t" PTDT_R16(8) PTDT_R16(4) PTDT_R16(2) PTDT_R16(1)
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]));
#undef PTDT_R16
  } else {
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = row16_sum(v[k]);
  }
}
// Packed fp32 (v_pk_fma_f32 / v_pk_mul_f32: two lanes' worth of FMAs per issue slot).
typedef float f2v __attribute__((ext_vector_type(2)));
// x . w over one feature chunk: even features accumulate in .x, odd ones in .y (one packed FMA per
// feature pair), then the halves are added -- exactly the scalar two-accumulator order
// (acc0 = x0 w0 + x2 w2 + ..., acc1 = x1 w1 + ..., acc0 + acc1).
template <int KP>
__device__ __forceinline__ float chunk_dot(const float (&x)[KP], const float (&w)[KP]) {
  f2v acc = {0.f, 0.f};
#pragma unroll
  for (int k = 0; k + 1 < KP; k += 2)
    acc = __builtin_elementwise_fma(f2v{x[k], x[k + 1]}, f2v{w[k], w[k + 1]}, acc);
  float a0 = acc.x;
  if constexpr ((KP & 1) != 0) a0 = fmaf(x[KP - 1], w[KP - 1], a0);
  return a0 + acc.y;
}
// SGD update kinds of the step loop (one loop instantiation each; no per-element branch)
constexpr int kSgdPlain = 0;  // no momentum, no weight decay: w -= lr * g (the reference's SGD(lr))
constexpr int kSgdNoMom = 1;  // weight decay, no momentum
constexpr int kSgdMom = 2;    // momentum (dampening, nesterov), weight decay
// raw buffer resource over [p, p + bytes): 32-bit offsets, out-of-range loads return 0
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// KP consecutive floats at byte offset `off` (dwordx4 / dwordx2 / dword pieces)
template <int KP>
__device__ __forceinline__ void buffer_load_chunk(__amdgpu_buffer_rsrc_t r, uint32_t off, float (&x)[KP]) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  int k = 0;
#pragma unroll
  for (; k + 4 <= KP; k += 4) {
    const f4v v = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(r, off + 4 * k, 0, 0));
    x[k] = v.x;
    x[k + 1] = v.y;
    x[k + 2] = v.z;
    x[k + 3] = v.w;
  }
  if constexpr (KP - (KP / 4) * 4 >= 2) {
    const f2v v = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(r, off + 4 * k, 0, 0));
    x[k] = v.x;
    x[k + 1] = v.y;
    k += 2;
  }
  if constexpr ((KP & 1) != 0) x[KP - 1] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off + 4 * (KP - 1), 0, 0));
}

template <int R, int KP, int DOUT, int LOSS, bool AR>
__global__ void __launch_bounds__(kThreads) linear_wave_f_kernel(FusedMlpArgs a, PersistArgs pa) {
  static_assert(R == 1 || R == 2 || R == 4, "rows per lane: 1, 2 or 4");
  // DOUT == 1: reduce-scatter, one row per lane (rows q & (R-1)); else every lane all rows
  constexpr bool SCATTER = DOUT == 1 && R > 1;
  constexpr int RY = SCATTER ? 1 : R;  // target rows a lane loads / computes the loss of
  extern __shared__ int elist[];
  // The kernel arguments the prologue reads are loaded here in one batch, pinned by the empty asm
  // (one wait for all), before the first branch. Left to the compiler, each scalar load followed
  // the branch it fed (stamps, timeline, start position, momentum, ...): five dependent kernel-
  // argument round trips before the first list load, and the start position came through a flat
  // load of a pointer selected between the cursor and the argument (round-5 kernel-entry asm).
  const int64_t r_now = (int64_t)__builtin_amdgcn_s_memrealtime();
  int64_t* const stamps_p = pa.stamps;
  int64_t* const tl_p = pa.tl;
  const int B = a.B, Din = a.Din, ns_arg = pa.num_samples, has_start = pa.has_start, start_e = pa.start_e,
            start_j = pa.start_j, has_bias_arg = a.has_bias, ldx_arg = a.ldx;
  const int32_t* const cursor_p = pa.cursor;
  const float* const P_arg = a.P;
  const float* const mom_arg = a.mom;
  const float* const X_arg = a.X;
  const float momentum_arg = a.momentum;
  asm volatile("" ::"s"(stamps_p), "s"(tl_p), "s"(B), "s"(Din), "s"(ns_arg), "s"(has_start), "s"(start_e), "s"(start_j),
               "s"(has_bias_arg), "s"(ldx_arg), "s"(cursor_p), "s"(P_arg), "s"(mom_arg), "s"(X_arg), "s"(momentum_arg));
  // diagnostic (stamps): kernel entry, for the prologue share of a launch (stamps[10], 10 ns ticks)
  const int64_t r_entry = stamps_p != nullptr ? r_now : 0;
  if (tl_p != nullptr && threadIdx.x == 0)  // tl_mark(tl, 0) with the entry time taken above
    __hip_atomic_store(tl_p, r_now, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int S = (ns_arg + B - 1) / B;
  // Lists are padded past num_samples with valid row indices (0): a batch's row slots rho * 16 + i
  // read their list entries unclamped (rows past the batch are masked by `valid`), so the last
  // batch may read up to (S - 1) * B + 16 R <= S * B + 64 entries. Same stride on the host (lds_bytes).
  const int estride = wave_list_stride(ns_arg, B);
  int e0 = start_e, j0 = start_j;
  if (!has_start) {  // the device cursor (plain launch): a load only on this path
    e0 = cursor_p[0];
    j0 = cursor_p[1];
  }
  const int64_t pos0 = (int64_t)e0 * S + j0;
  const int n = pa.n_steps;
  const int T = (j0 + n - 1) / S;  // epoch barriers crossed (j0 < S)
  auto list = [&](int e) { return elist + (e & 1) * estride; };
  // diagnostic prologue split (stamps[11..13], 10 ns ticks): position known, list in LDS, after the barrier
  int64_t r_pro[3] = {0, 0, 0};
  auto pstamp = [&](int k) {
    if (stamps_p != nullptr) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      r_pro[k] = (int64_t)__builtin_amdgcn_s_memrealtime();
    }
  };
  pstamp(0);

  // Only the first epoch's list is on the path to step 0. The next one is
  // zero-filled (row 0: the trainer reads stale-but-valid indices for the kNB
  // positions past its last step, so every entry it can touch must be a valid
  // dataset row -- no clamp per load) and built by the helper waves after the
  // barrier, while the trainer runs epoch e0.
  // With a list cache (pa.lcache) a launch that starts inside an already
  // computed epoch copies its list instead of recomputing the permutation.
  // The trainer wave's parameters and momenta are read first: their latency
  // overlaps the epoch list's (both on the path to step 0).
  const int lane = (int)threadIdx.x;
  const int q = (lane & 63) >> 4, i = lane & 15;  // feature group, row slot
  const int k0 = q * KP;
  const bool hb = has_bias_arg != 0;
  const bool use_mom = mom_arg != nullptr && momentum_arg != 0.f;
  const int nW = DOUT * Din;
  float W[DOUT][KP], M[DOUT][KP], Wb[DOUT], Mb[DOUT];
  if (wave == 0) {
    const auto P = gptr(P_arg);
#pragma unroll
    for (int c = 0; c < DOUT; ++c) {
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        const bool in = k0 + k < Din;
        W[c][k] = in ? P[c * Din + k0 + k] : 0.f;
        M[c][k] = (in && use_mom) ? gptr(mom_arg)[c * Din + k0 + k] : 0.f;
      }
      Wb[c] = hb ? P[nW + c] : 0.f;
      Mb[c] = (hb && use_mom) ? gptr(mom_arg)[nW + c] : 0.f;
    }
  }
  // batch loads: x rows of this lane's feature group, the targets of its loss rows
  const int rho_own = SCATTER ? (q & (R - 1)) : 0;  // the row whose loss this lane computes
  const int ldx = ldx_arg > 0 ? ldx_arg : Din;  // feature slots past Din read X's zero padding
  // Gathers through buffer resources with 32-bit byte offsets (the host checks N * ldx * 4 < 2^31,
  // sel, ldx * 4 < 2^24): one v_mad_u32_u24 per row instead of a 64-bit address chain.
  const uint32_t n_rows = (uint32_t)pa.N;
  const __amdgpu_buffer_rsrc_t xrs = buffer_rsrc(X_arg, n_rows * (uint32_t)ldx * 4u);
  const __amdgpu_buffer_rsrc_t yrs =
      LOSS == kLossCEIndex ? buffer_rsrc(a.Yi, n_rows * 8u) : buffer_rsrc(a.Yf, n_rows * (uint32_t)(DOUT * 4));
  const uint32_t ldx4 = (uint32_t)ldx * 4u, k04 = (uint32_t)k0 * 4u;
  // loss scales of a full batch and of the one short last batch (nb_last == B if none); each batch
  // carries its pair, selected at fetch time (off the step's dependent chain)
  const int nb_last = ns_arg - (S - 1) * B;
  const float inv_full = 1.f / (float)((LOSS == kLossMSE) ? B * DOUT : B);
  const float inv_last = 1.f / (float)((LOSS == kLossMSE) ? nb_last * DOUT : nb_last);
  const float gs_full = a.grad_scale * inv_full, gs_last = a.grad_scale * inv_last;
  auto load_batch = [&](Batch<R, KP, DOUT, RY>& f, const int (&sel)[R], int sel_y, int nb) {
    f.nb = nb;
    f.cg = nb == B ? gs_full : gs_last;
    f.cl = nb == B ? inv_full : inv_last;
#pragma unroll
    for (int rho = 0; rho < R; ++rho) buffer_load_chunk<KP>(xrs, __umul24((uint32_t)sel[rho], ldx4) + k04, f.x[rho]);
#pragma unroll
    for (int ry = 0; ry < RY; ++ry) {
      const uint32_t s = (uint32_t)(SCATTER ? sel_y : sel[ry]);
      if constexpr (LOSS == kLossCEIndex) {
        f.yi[ry] = __builtin_amdgcn_raw_buffer_load_b32(yrs, s * 8u, 0, 0);  // low dword (see mlp_tp.hip)
      } else {
#pragma unroll
        for (int c = 0; c < DOUT; ++c)
          f.y[ry][c] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(yrs, s * (uint32_t)(DOUT * 4) + 4u * c, 0, 0));
      }
    }
  };
  Batch<R, KP, DOUT, RY> buf[kNB];
  const ListCache lc{pa.lcache, pa.ltag, al4(ns_arg)};  // the global cache keeps the unpadded stride
  rank_epoch_indices_or(given_list(pa, e0), list(e0), (uint32_t)pa.N, pa.W, pa.rank, pa.num_samples, pa.seed, e0, pa.shuffle,
                     (int)threadIdx.x, kThreads, lc);
  for (int k = (int)threadIdx.x; k < estride; k += kThreads) list(e0 + 1)[k] = 0;
  for (int k = ns_arg + (int)threadIdx.x; k < estride; k += kThreads) list(e0)[k] = 0;  // builders write [0, ns)
  pstamp(1);
  // Loss ring (pa.loss_ring): the trainer stores each lane's scaled loss share
  // per step (one ds_write), the helper waves add the 64 shares and write
  // losses[] -- the per-step cross-lane loss reduction leaves the critical path.
  const int ring = pa.loss_ring ? 2 * S + kNB : 0;  // slots; 2 epochs + prefetch depth never overwrite unread
  float* const lring = reinterpret_cast<float*>(elist + 2 * estride + 16);  // after the 8 u64 timer slots
  __syncthreads();
  pstamp(2);
  tl_mark(pa.tl, 1);
  if (wave != 0) {
    const int ht = (int)threadIdx.x - 64, hn = kThreads - 64;
    int64_t lo = pos0;
    // positions [lo, hi): 16 lanes per position (a DPP row), 4 shares per lane (one 16-B LDS read),
    // then a fixed-order 16-lane tree -- the final call runs after the last step, in the launch's tail
    // (a progressive variant -- the helpers polling a trainer step count in LDS and reducing each
    // position as it completed -- cost 0.017 us per step and did not shorten the tail; round 6)
    auto reduce_losses = [&](int64_t hi) {
      const int grp = ht >> 4, sub = ht & 15, ngrp = hn >> 4;
      for (int64_t P = lo + grp; P < hi; P += ngrp) {
        const float* sh = lring + ((int)(P - pos0) % ring) * 64;
        const float4 v = *reinterpret_cast<const float4*>(sh + 4 * sub);
        const float acc = group_sum<16>((v.x + v.y) + (v.z + v.w));
        if (sub == 0) pa.losses[P - pos0] = acc;
      }
      lo = hi > lo ? hi : lo;
    };
    if (ht == 0 && pa.idx == nullptr) list_cache_publish(lc, e0);  // every thread's entries written (barrier)
    if (T > 0)  // epoch e0+1, needed at the trainer's first barrier
      rank_epoch_indices_or(given_list(pa, e0 + 1), list(e0 + 1), (uint32_t)pa.N, pa.W, pa.rank, pa.num_samples, pa.seed, e0 + 1,
                            pa.shuffle, ht, hn, lc);
    for (int i = 1; i <= T; ++i) {
      __syncthreads();
      if (ht == 0 && pa.idx == nullptr) list_cache_publish(lc, e0 + i);  // built before barrier i
      if (i < T)
        rank_epoch_indices_or(given_list(pa, e0 + i + 1), list(e0 + i + 1), (uint32_t)pa.N, pa.W, pa.rank, pa.num_samples, pa.seed, e0 + i + 1,
                           pa.shuffle, ht, hn, lc);
      // at barrier i the trainer has trained every position before (e0+i)*S - kNB
      if (ring) reduce_losses(min((int64_t)(e0 + i) * S - kNB, pos0 + n));
    }
    if (ring) {
      __syncthreads();  // the trainer's final barrier: every step done
      reduce_losses(pos0 + n);
    }
    return;
  }

  const float lr = a.lr, mu = a.momentum, damp = a.dampening, wd = a.weight_decay;
  const int nesterov = a.nesterov;

  int opt_step = a.opt_step ? *a.opt_step : 0;
  const XgmiArgs& ar = a.ar;
  const int world = AR ? ar.world : 1;
  uint64_t PTDT_GLOBAL* push_dst = nullptr;  // row slot i pushes to rank i
#pragma unroll
  for (int r = 0; r < kXgmiMaxRanks; ++r)
    if (i == r && r < world) push_dst = (uint64_t PTDT_GLOBAL*)ar.peers[r];
  uint64_t PTDT_GLOBAL* const poll_src = (uint64_t PTDT_GLOBAL*)ar.local;
  const int my_rank = ar.rank, max_elems = ar.max_elems;
  float PTDT_GLOBAL* const losses = gptr_w(pa.losses);
  uint32_t seq = AR ? *ar.seq : 0u;
  bool failed = AR && *ar.err != 0;
  const float inv_w = 1.f / (float)world;
  // world 2: one packed store + one poll per step (ll_exchange_pair), staged through 128 LDS floats
  __shared__ float xpair[AR ? 128 : 1];
  const bool pair = AR && world == 2 && (ar.flags & kXgmiPair) != 0u && DOUT * (Din + 1) <= 64;

  int ie = e0, ij = j0, barriers = 0;
  int sel_next[R], sel_y_next = 0, nb_next = 0;
  // running LDS entry offset of position (ie, ij) and a barrier owed by the last epoch wrap: the
  // per-step bookkeeping is an add and a compare (it was the list base, ij * B and the three-way
  // barrier condition recomputed every step)
  int lofs = (ie & 1) * estride + ij * B;
  bool bar_due = false;
  auto read_index = [&]() {
    if (bar_due) {  // new epoch: its list is ready, the old one free
      __syncthreads();
      ++barriers;
      bar_due = false;
    }
    nb_next = ij == S - 1 ? nb_last : B;
#pragma unroll
    for (int rho = 0; rho < R; ++rho) sel_next[rho] = elist[lofs + rho * 16 + i];
    if constexpr (SCATTER)  // own row's index read directly: selecting from sel_next[] by a lane value spills it
      sel_y_next = elist[lofs + rho_own * 16 + i];
    lofs += B;
    if (++ij == S) {
      ij = 0;
      ++ie;
      lofs = (ie & 1) * estride;
      bar_due = barriers < T;
    }
  };
  auto fetch = [&](Batch<R, KP, DOUT, RY>& f) {
    load_batch(f, sel_next, sel_y_next, nb_next);
    read_index();
  };

  Ticks tk;
  tk.on = pa.stamps != nullptr;
  tk.acc = reinterpret_cast<unsigned long long*>(elist + 2 * estride);
  if (tk.on && lane == 0)
    for (int k = 0; k < 8; ++k) tk.acc[k] = 0ull;
  const int64_t t_begin = tk.on ? (int64_t)__builtin_amdgcn_s_memtime() : 0;
  const int64_t r_begin = tk.on ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;

  auto row_loss = [&](const float* z, const float* y, int yi, bool valid, float* g, float& l, float& cnt) {
    l = 0.f;
    cnt = 0.f;
    if constexpr (LOSS == kLossMSE) {
#pragma unroll
      for (int c = 0; c < DOUT; ++c) {
        const float df = z[c] - y[c];
        l = fmaf(df, df, l);
        g[c] = 2.f * df;
      }
    } else if constexpr (DOUT == 1) {
      const float ls0 = z[0] - z[0];  // log_softmax of one class: 0 (NaN if z is not finite)
      if constexpr (LOSS == kLossCESoft) {
        l = -y[0] * ls0;
        g[0] = fmaf(ls0, y[0], 0.f);  // exp(ls0) y - y: the same bits (+0, or NaN), one op shorter
      } else {
        const bool use = yi != a.ignore_index;
        g[0] = use ? (ls0 + 1.f) - (yi == 0 ? 1.f : 0.f) : 0.f;
        l = use ? -(yi == 0 ? ls0 : 0.f) : 0.f;
        cnt = use ? 1.f : 0.f;
      }
    } else {
      float m = z[0];
#pragma unroll
      for (int c = 1; c < DOUT; ++c) m = fmaxf(m, z[c]);
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < DOUT; ++c) se += __expf(z[c] - m);
      const float lse = m + __builtin_amdgcn_logf(se) * 0.6931471805599453f;
      if constexpr (LOSS == kLossCESoft) {
        float tsum = 0.f;
#pragma unroll
        for (int c = 0; c < DOUT; ++c) {
          tsum += y[c];
          l -= y[c] * (z[c] - lse);
        }
#pragma unroll
        for (int c = 0; c < DOUT; ++c) g[c] = __expf(z[c] - lse) * tsum - y[c];
      } else {
        const bool use = yi != a.ignore_index;
        float zy = 0.f;
#pragma unroll
        for (int c = 0; c < DOUT; ++c) {
          zy = c == yi ? z[c] : zy;
          g[c] = use ? __expf(z[c] - lse) - (c == yi ? 1.f : 0.f) : 0.f;
        }
        l = use ? lse - zy : 0.f;
        cnt = use ? 1.f : 0.f;
      }
    }
    if (!valid) {
#pragma unroll
      for (int c = 0; c < DOUT; ++c) g[c] = 0.f;
      l = 0.f;
      cnt = 0.f;
    }
  };

  float Gk[DOUT][KP], Gbk[DOUT];
#pragma unroll
  for (int c = 0; c < DOUT; ++c) {
    Gbk[c] = 0.f;
#pragma unroll
    for (int k = 0; k < KP; ++k) Gk[c][k] = 0.f;
  }
  int rslot = 0;  // loss ring slot of the next step
  const float lr_b = hb ? lr : 0.f;  // plain SGD's bias step
  auto train = [&](Batch<R, KP, DOUT, RY>& f, int step, auto sgd_tag, auto ring_tag) {
    constexpr int SGD = decltype(sgd_tag)::value;
    constexpr bool MOM = SGD == kSgdMom;
    constexpr bool RING = decltype(ring_tag)::value;
    const int nb = f.nb;
    // ---- forward: partial logits of this feature group
    float zp[R][DOUT];
#pragma unroll
    for (int rho = 0; rho < R; ++rho) {
#pragma unroll
      for (int c = 0; c < DOUT; ++c) zp[rho][c] = chunk_dot<KP>(f.x[rho], W[c]);
    }
    tk.tick(1);
    // ---- logits -> loss -> dL/dz (g[rho][c] in every lane)
    float g[R][DOUT], lsum, csum;
    if constexpr (SCATTER) {
      float z;
      if constexpr (R == 2) {
        const float s = rs16(zp[0][0], zp[1][0]);
        z = rs32(s, s);  // DPP rows {0,2}: batch row 0, {1,3}: batch row 1
      } else {
        z = rs32(rs16(zp[0][0], zp[1][0]), rs16(zp[2][0], zp[3][0]));  // DPP row q: batch row q
      }
      z += Wb[0];
      float gz, l, cnt;
      row_loss(&z, f.y[0], f.yi[0], rho_own * 16 + i < nb, &gz, l, cnt);
      // each batch row counted once: R == 2 has every row in two DPP rows
      const bool owner = R == 4 || q < 2;
      lsum = owner ? l : 0.f;
      csum = owner ? cnt : 0.f;
      if constexpr (LOSS != kLossCEIndex) gz *= f.cg;  // 1/B once
      if constexpr (R == 2) {
        const F2 r = pl16(gz, gz);  // rows [g0, g0, g0, g0], [g1, g1, g1, g1]
        g[0][0] = r.a;
        g[1][0] = r.b;
      } else {
        const F2 h = pl32(gz, gz);   // [g0, g1, g0, g1], [g2, g3, g2, g3]
        const F2 r01 = pl16(h.a, h.a);
        const F2 r23 = pl16(h.b, h.b);
        g[0][0] = r01.a;
        g[1][0] = r01.b;
        g[2][0] = r23.a;
        g[3][0] = r23.b;
      }
    } else {
      lsum = 0.f;
      csum = 0.f;
#pragma unroll
      for (int rho = 0; rho < R; ++rho) {
        float z[DOUT];
#pragma unroll
        for (int c = 0; c < DOUT; ++c) z[c] = allrows(zp[rho][c]) + Wb[c];
        float l, cnt;
        row_loss(z, f.y[rho], f.yi[rho], rho * 16 + i < nb, g[rho], l, cnt);
        lsum += l;
        csum += cnt;
      }
      if (q != 0) {  // the 4 DPP rows computed the same rows: count them once
        lsum = 0.f;
        csum = 0.f;
      }
    }
    float inv_denom;
    if constexpr (LOSS == kLossCEIndex) {
      csum = wave_sum(csum);
      inv_denom = 1.f / (csum > 0.f ? csum : 1.f);
    } else {
      inv_denom = f.cl;
    }
    // SCATTER already applied the scale to dL/dz before the all-gather
    const float coef = (SCATTER && LOSS != kLossCEIndex) ? 1.f : a.grad_scale * inv_denom;
    tk.tick(2);
    // ---- backward: column sums over the 16 row slots of this DPP row
    float gW[DOUT][KP], gb[DOUT];
#pragma unroll
    for (int c = 0; c < DOUT; ++c) {
      // sum over the lane's rows, feature pairs packed: t = g0 x0 + g1 x1 + ... (scalar order)
      float t[KP];
#pragma unroll
      for (int k = 0; k + 1 < KP; k += 2) {
        f2v tv = f2v{f.x[0][k], f.x[0][k + 1]} * f2v{g[0][c], g[0][c]};
#pragma unroll
        for (int rho = 1; rho < R; ++rho)
          tv = __builtin_elementwise_fma(f2v{f.x[rho][k], f.x[rho][k + 1]}, f2v{g[rho][c], g[rho][c]}, tv);
        t[k] = tv.x;
        t[k + 1] = tv.y;
      }
      if constexpr ((KP & 1) != 0) {
        float tl = g[0][c] * f.x[0][KP - 1];
#pragma unroll
        for (int rho = 1; rho < R; ++rho) tl = fmaf(g[rho][c], f.x[rho][KP - 1], tl);
        t[KP - 1] = tl;
      }
      float tb = g[0][c];
#pragma unroll
      for (int rho = 1; rho < R; ++rho) tb += g[rho][c];
      // the KP weight sums and the bias sum of class c: one row16_sum_n group
      float sums[KP + 1];
#pragma unroll
      for (int k = 0; k < KP; ++k) sums[k] = t[k];
      sums[KP] = tb;
      row16_sum_n<KP + 1>(sums);
#pragma unroll
      for (int k = 0; k < KP; ++k) gW[c][k] = (SCATTER && LOSS != kLossCEIndex) ? sums[k] : sums[k] * coef;
      gb[c] = (SCATTER && LOSS != kLossCEIndex) ? sums[KP] : sums[KP] * coef;
    }
    tk.tick(3);
    // ---- all-reduce over ranks: row slot r <-> rank r, summed with the same DPP tree
    if (AR && !failed && pair) {
      seq += 1u;
      failed = !ll_exchange_pair<KP, DOUT>(ar, seq, q, i, lane, Din, gW, gb, xpair, inv_w,
                                           ar.drop_push != 0u && seq >= ar.drop_push);
      failed = __any(failed);
    } else if (AR && !failed) {
      seq += 1u;
      float v[DOUT][KP], vb[DOUT];
#pragma unroll
      for (int c = 0; c < DOUT; ++c) {  // own contribution from registers, slots >= world add 0
        vb[c] = i == my_rank ? gb[c] : 0.f;
#pragma unroll
        for (int k = 0; k < KP; ++k) v[c][k] = i == my_rank ? gW[c][k] : 0.f;
      }
      // (ll_exchange_u / ll_exchange_packed / a separate pusher or poller wave measured no faster at
      //  W = 8: tools/exchange_bench.hip, profiles/r3_exchange_bench*.jsonl; W = 2 takes the pair path)
      const bool ok = ll_exchange<KP, DOUT>(i < world && i != my_rank, push_dst, poll_src, my_rank, i, world,
                                            max_elems, seq, k0, Din, hb, q == 0, 4 * KP != Din, gW, gb, v, vb,
                                            ar.err, ar.max_polls, ar.drop_push != 0u && seq >= ar.drop_push);
      failed = !ok;
      failed = __any(failed);
#pragma unroll
      for (int c = 0; c < DOUT; ++c) {  // the ranks' sum: the same DPP tree (row16_sum_n group per class)
        float sums[KP + 1];
#pragma unroll
        for (int k = 0; k < KP; ++k) sums[k] = v[c][k];
        sums[KP] = vb[c];
        row16_sum_n<KP + 1>(sums);
#pragma unroll
        for (int k = 0; k < KP; ++k) gW[c][k] = sums[k] * inv_w;
        gb[c] = sums[KP] * inv_w;
      }
    }
    tk.tick(4);
    // ---- SGD on this lane's feature group (SGD: the update kind; the caller
    // instantiates the whole step loop per kind, so no per-step branch)
    const bool first = opt_step == 0;
    auto upd = [&](float& w, float& m, float gr) {
      if constexpr (SGD == kSgdPlain) {  // d = g + 0 * w == g for every finite w
        w = fmaf(-lr, gr, w);
        return;
      }
      float d = fmaf(wd, w, gr);
      if constexpr (MOM) {
        const float buf = first ? d : fmaf(mu, m, (1.f - damp) * d);
        m = buf;
        d = nesterov ? fmaf(mu, buf, d) : buf;
      }
      w = fmaf(-lr, d, w);
    };
#pragma unroll
    for (int c = 0; c < DOUT; ++c) {
#pragma unroll
      for (int k = 0; k < KP; ++k) upd(W[c][k], M[c][k], gW[c][k]);
      if constexpr (SGD == kSgdPlain) {
        Wb[c] = fmaf(-lr_b, gb[c], Wb[c]);  // no bias: lr_b = 0 keeps Wb at 0 (no select)
      } else {
        upd(Wb[c], Mb[c], gb[c]);
        Wb[c] = hb ? Wb[c] : 0.f;
      }
    }
    ++opt_step;
    // the DDP bucket (a.G) keeps the last step's averaged gradients: register
    // copies here (the unrolled loop keeps only the last), one store at the end
#pragma unroll
    for (int c = 0; c < DOUT; ++c) {
#pragma unroll
      for (int k = 0; k < KP; ++k) Gk[c][k] = gW[c][k];
      Gbk[c] = gb[c];
    }
    // ---- loss report
    if constexpr (RING) {  // this lane's share; the helper waves add the 64 shares
      const float share = (LOSS == kLossCEIndex && !(csum > 0.f)) ? NAN : lsum * inv_denom;
      lring[rslot * 64 + lane] = share;
      rslot = rslot + 1 == ring ? 0 : rslot + 1;
    } else {  // row sums by DPP, the 4 DPP rows by two swaps
      const float ls = allrows(row16_sum(lsum));
      if constexpr (LOSS == kLossCEIndex) losses[step] = csum > 0.f ? ls * inv_denom : NAN;
      else losses[step] = ls * inv_denom;
    }
    tk.tick(5);
  };

  tk.start();
  read_index();
#pragma unroll
  for (int u = 0; u < kNB; ++u) fetch(buf[u]);
  tk.tick(0);
  int done = 0;
  const int nfull = n - n % kNB;
  auto run = [&](auto sgd_tag, auto ring_tag) {
    while (done < nfull && !failed) {
#pragma unroll
      for (int u = 0; u < kNB; ++u) {
        train(buf[u], done + u, sgd_tag, ring_tag);
        fetch(buf[u]);
        tk.tick(0);
      }
      done += kNB;
    }
#pragma unroll
    for (int u = 0; u < kNB - 1; ++u) {
      if (done < n && !failed) {
        train(buf[u], done, sgd_tag, ring_tag);
        ++done;
      }
    }
  };
  // one loop instantiation per (SGD kind, loss ring): no per-step branch on either. Plain SGD (the
  // reference's SGD(lr)) has its own loop with the ring only; without the ring it takes the
  // weight-decay loop (same values: d = g + 0 * w).
  using Plain = std::integral_constant<int, kSgdPlain>;
  using NoMom = std::integral_constant<int, kSgdNoMom>;
  using Mom = std::integral_constant<int, kSgdMom>;
  if (use_mom) {
    if (ring) run(Mom{}, std::true_type{});
    else run(Mom{}, std::false_type{});
  } else if (ring) {
    if (wd == 0.f) run(Plain{}, std::true_type{});
    else run(NoMom{}, std::true_type{});
  } else {
    run(NoMom{}, std::false_type{});
  }
  tl_mark(pa.tl, 2);
  // final stores first, then the remaining barriers: their latency overlaps the helpers' tail
  if (i == 0) {
    const auto Pw = gptr_w(a.P);
    const auto Gw = gptr_w(a.G);
#pragma unroll
    for (int c = 0; c < DOUT; ++c) {
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        if (k0 + k < Din) {
          Pw[c * Din + k0 + k] = W[c][k];
          if (done > 0) Gw[c * Din + k0 + k] = Gk[c][k];
          if (use_mom) a.mom[c * Din + k0 + k] = M[c][k];
        }
      }
      if (hb && q == 0) {
        Pw[nW + c] = Wb[c];
        if (done > 0) Gw[nW + c] = Gbk[c];
        if (use_mom) a.mom[nW + c] = Mb[c];
      }
    }
  }
  if (lane == 0) {
    const int64_t pos = pos0 + done;
    pa.cursor[0] = (int)(pos / S);
    pa.cursor[1] = (int)(pos % S);
    if (a.opt_step) *a.opt_step = opt_step;
    if (AR) *ar.seq = seq;
    if (tk.on) {
      for (int k = 0; k < 6; ++k) pa.stamps[k] += (int64_t)tk.acc[k];
      pa.stamps[7] += (int64_t)__builtin_amdgcn_s_memtime() - t_begin;
      pa.stamps[8] += (int64_t)__builtin_amdgcn_s_memrealtime() - r_begin;
      pa.stamps[10] += r_begin - r_entry;
      if (pa.stamps_n >= 14) {
        pa.stamps[11] += r_pro[0] - r_entry;
        pa.stamps[12] += r_pro[1] - r_pro[0];
        pa.stamps[13] += r_pro[2] - r_pro[1];
      }
    }
  }
  while (barriers < T) {
    __syncthreads();
    ++barriers;
  }
  if (ring) __syncthreads();  // final barrier: the helpers reduce the remaining losses
  if (pa.tl != nullptr) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // the final stores issued above are done
    tl_mark(pa.tl, 3);
  }
}

// Instantiation table of one loss and all-reduce flag: (L, R, KP, DOUT)
// combinations whose register footprint fits (no scratch). nullptr otherwise.
// Keep in sync with kWaveConfigs in linear_wave.hip.
// L == 0 selects layout F (linear_wave_f_kernel), R in {1, 2, 4}.
template <int LOSS, bool AR>
const void* pick(int L, int R, int kp, int dout) {
#define PTDT_LWF(RR, KP, DO) \
  if (L == 0 && R == RR && kp == KP && dout == DO) return (const void*)linear_wave_f_kernel<RR, KP, DO, LOSS, AR>;
#define PTDT_LWF_R(RR)                                                                             \
  PTDT_LWF(RR, 4, 1) PTDT_LWF(RR, 5, 1) PTDT_LWF(RR, 8, 1) PTDT_LWF(RR, 10, 1) PTDT_LWF(RR, 16, 1) \
  PTDT_LWF(RR, 4, 2) PTDT_LWF(RR, 5, 2) PTDT_LWF(RR, 8, 2)
  PTDT_LWF_R(1) PTDT_LWF_R(2) PTDT_LWF_R(4)
#undef PTDT_LWF_R
#undef PTDT_LWF
#define PTDT_LW(LL, RR, KP, DO) \
  if (L == LL && R == RR && kp == KP && dout == DO) return (const void*)linear_wave_kernel<LL, RR, KP, DO, LOSS, AR>;
#define PTDT_LW_LR(LL, RR)                                                                    \
  PTDT_LW(LL, RR, 4, 1) PTDT_LW(LL, RR, 5, 1) PTDT_LW(LL, RR, 8, 1) PTDT_LW(LL, RR, 10, 1)    \
  PTDT_LW(LL, RR, 16, 1) PTDT_LW(LL, RR, 4, 2) PTDT_LW(LL, RR, 5, 2) PTDT_LW(LL, RR, 8, 2)    \
  PTDT_LW(LL, RR, 10, 2) PTDT_LW(LL, RR, 4, 4)
  PTDT_LW_LR(1, 1) PTDT_LW_LR(2, 1) PTDT_LW_LR(4, 1) PTDT_LW_LR(8, 1) PTDT_LW_LR(2, 2) PTDT_LW_LR(4, 2)
#undef PTDT_LW_LR
#undef PTDT_LW
  return nullptr;
}

}  // namespace lw
}  // namespace ptdt
