// Microbenchmark: the single-wave engine's per-step gradient exchange in isolation.
// `world` workgroups of one wave each play the ranks of one GPU (each its own region of
// one uncached LL buffer, as XgmiComm allocates it); every iteration a dependent chain
// of `work` FMAs stands for the step's forward/loss/backward, then the layout-F chunk
// (KP = 5 weights + bias per lane, Linear(20, 1)) is exchanged and summed over the row
// slots (row16_sum), and the sum feeds the next iteration -- the engine's critical path.
// Variants: 0 = ll_exchange (round-2 protocol), 1 = ll_exchange_u (uniform poll loop,
// two batches in flight), 2 = a second wave pushes (the chunk handed over through LDS) so
// the training wave's polls never queue behind its own stores (vmcnt counts loads and
// stores in order on gfx9), 3 = a second wave polls and sums (every rank self-pushes) and
// hands the sum back through LDS, so the training wave never waits for a poll round trip
// after its stores, 4 = the rank's 21 values as 21 consecutive words (one store and one poll
// instruction per peer, LDS redistribution; peers polled one after another), 5 = one word per
// peer (the protocol's floor), 6 = packed as 4 with every peer's stores and polls in flight
// together (lane f: peer f / 21, word f % 21) and the rank-order sums read from LDS.
// Prints cycles (s_memtime) per iteration and checks that every rank ends with identical weights.
// Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -Icsrc tools/exchange_bench.hip -o tools/bin/exchange_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "kernels/linear_wave_impl.h"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

using namespace ptdt;
constexpr int KP = 5, DOUT = 1, DIN = 20;

template <int VARIANT>
__global__ void __launch_bounds__(128) k_exchange(uint64_t* buf, int world, int max_elems, int iters, int work,
                                                  int* err, long long* cycles, float* out) {
  __shared__ float hand[2][64 * (KP + 1)];  // per-parity hand-over / staging (variants 2-6)
  const int rank = blockIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = threadIdx.x & 63, q = lane >> 4, i = lane & 15, k0 = q * KP;
  const int64_t region = (int64_t)2 * world * max_elems;
  uint64_t PTDT_GLOBAL* const local = (uint64_t PTDT_GLOBAL*)(buf + rank * region);
  uint64_t PTDT_GLOBAL* push_dst = nullptr;
#pragma unroll
  for (int r = 0; r < kXgmiMaxRanks; ++r)
    if (i == r && r < world) push_dst = (uint64_t PTDT_GLOBAL*)(buf + r * region);
  const float inv_w = 1.f / (float)world;
  if (wave == 1) {  // helper wave of variants 2 / 3
    if (VARIANT < 2 || VARIANT > 3 || world == 1) return;  // (4-6: single wave)
    const float zero[1][KP] = {}, zb[1] = {};
    for (uint32_t seq = 1; seq <= (uint32_t)iters; ++seq) {
      float* h = hand[seq & 1];
      if constexpr (VARIANT == 2) {  // pusher: the chunk arrives through LDS after the barrier
        __builtin_amdgcn_s_barrier();
        float gW[1][KP], gb[1];
#pragma unroll
        for (int k = 0; k < KP; ++k) gW[0][k] = h[lane * (KP + 1) + k];
        gb[0] = h[lane * (KP + 1) + KP];
        if (i < world && i != rank)
          lw::ll_push_chunk<KP, DOUT>(push_dst, rank, world, max_elems, seq, k0, DIN, true, q == 0, false, gW, gb);
      } else {  // poller: every slot from memory (self-pushed), sum, hand back, barrier
        float v[1][KP], vb[1];
        lw::ll_poll_chunk<KP, DOUT>(local, rank, i, world, max_elems, seq, k0, DIN, true, true, zero, zb, v, vb, err,
                                    1u << 20);
#pragma unroll
        for (int k = 0; k < KP; ++k) h[lane * (KP + 1) + k] = lw::row16_sum(v[0][k]) * inv_w;
        h[lane * (KP + 1) + KP] = lw::row16_sum(vb[0]) * inv_w;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
    }
    return;
  }
  float x = 1.f + 0.001f * (float)lane + 0.01f * (float)rank;  // rank-dependent data, the same weights:
  float W[KP];                                                    // replicas stay equal only via the all-reduce
#pragma unroll
  for (int k = 0; k < KP; ++k) W[k] = 0.1f * (float)(k0 + k);
  uint32_t seq = 0;
  bool failed = false;
  const long long t0 = (long long)__builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters && !failed; ++it) {
    // the step's compute: a dependent chain on this lane's chunk
    float acc = x;
    for (int w = 0; w < work; ++w) acc = fmaf(acc, 0.999f, W[0] * 1e-3f);
    float gW[DOUT][KP], gb[DOUT];
#pragma unroll
    for (int k = 0; k < KP; ++k) gW[0][k] = lw::row16_sum((acc + W[k]) * (float)(k + 1) * 1e-3f);
    gb[0] = lw::row16_sum(acc * 1e-3f);
    if (world > 1) {
      seq += 1u;
      float v[DOUT][KP], vb[DOUT];
      bool ok = true;
      if constexpr (VARIANT == 0) {
#pragma unroll
        for (int k = 0; k < KP; ++k) v[0][k] = i == rank ? gW[0][k] : 0.f;
        vb[0] = i == rank ? gb[0] : 0.f;
        ok = lw::ll_exchange<KP, DOUT>(i < world && i != rank, push_dst, local, rank, i, world, max_elems, seq, k0,
                                       DIN, true, q == 0, false, gW, gb, v, vb, err, 1u << 20, false);
      } else if constexpr (VARIANT == 1) {
        ok = lw::ll_exchange_u<KP, DOUT>(i < world && i != rank, push_dst, local, rank, i, world, max_elems, seq, k0,
                                         DIN, true, q == 0, false, gW, gb, v, vb, err, 1u << 20);
      } else if constexpr (VARIANT == 2) {  // hand the chunk to the pusher, poll right away
        float* h = hand[seq & 1];
#pragma unroll
        for (int k = 0; k < KP; ++k) h[lane * (KP + 1) + k] = gW[0][k];
        h[lane * (KP + 1) + KP] = gb[0];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        ok = lw::ll_poll_chunk<KP, DOUT>(local, rank, i, world, max_elems, seq, k0, DIN, true, false, gW, gb, v, vb,
                                         err, 1u << 20);
      }
      if constexpr (VARIANT == 6) {
        // packed, every peer in parallel: the rank's 21 values are staged in LDS, lane f of the
        // push/poll instructions handles (peer f / 21, word f % 21) -- 21 consecutive words per
        // peer, all peers' stores and polls in flight together -- and each lane then sums its
        // chunk's 6 words over the ranks (rank order) from LDS
        constexpr int NPW = 21;
        const int parity = (int)(seq & 1u);
        const uint64_t hi = (uint64_t)seq << 32;
        float* stg = hand[seq & 1];                 // [21] own values
        float* pol = hand[seq & 1] + 32;            // [world][21] every rank's values (rank order)
        if (i == 0) {
#pragma unroll
          for (int k = 0; k < KP; ++k) stg[q * KP + k] = gW[0][k];
          if (q == 0) stg[20] = gb[0];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int npeer = world - 1;
        const int nf = NPW * npeer;                 // <= 147 for world 8: 3 instructions
        float own[3];
        int pr[3], wd[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          const int f = lane + 64 * t;
          const int pi = f / NPW;
          wd[t] = f - pi * NPW;
          pr[t] = f < nf ? (pi < rank ? pi : pi + 1) : -1;
          own[t] = stg[wd[t]];
        }
#pragma unroll
        for (int t = 0; t < 3; ++t)
          if (pr[t] >= 0) {
            uint64_t PTDT_GLOBAL* dst =
                (uint64_t PTDT_GLOBAL*)(buf + pr[t] * region) + (int64_t)(parity * world + rank) * max_elems + wd[t];
            __hip_atomic_store(dst, hi | __float_as_uint(own[t]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
        uint64_t w[3];
        auto issue = [&]() {
#pragma unroll
          for (int t = 0; t < 3; ++t) {
            const int src = pr[t] >= 0 ? pr[t] : (rank + 1 == world ? 0 : rank + 1);
            w[t] = __hip_atomic_load(local + (int64_t)(parity * world + src) * max_elems + (pr[t] >= 0 ? wd[t] : 0),
                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
        };
        issue();
        for (uint32_t n = 0; n < (1u << 20); ++n) {
          bool m = false;
#pragma unroll
          for (int t = 0; t < 3; ++t) m |= pr[t] >= 0 && (uint32_t)(w[t] >> 32) != seq;
          if (__builtin_amdgcn_ballot_w64(m) == 0) break;
          issue();
        }
#pragma unroll
        for (int t = 0; t < 3; ++t)
          if (pr[t] >= 0) pol[pr[t] * NPW + wd[t]] = __uint_as_float((uint32_t)w[t]);
        if (lane < NPW) pol[rank * NPW + lane] = stg[lane];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        float sw[KP], sb = 0.f;
#pragma unroll
        for (int k = 0; k < KP; ++k) sw[k] = 0.f;
        for (int p = 0; p < world; ++p) {  // rank order: identical bits on every rank
#pragma unroll
          for (int k = 0; k < KP; ++k) sw[k] += pol[p * NPW + q * KP + k];
          sb += pol[p * NPW + 20];
        }
#pragma unroll
        for (int k = 0; k < KP; ++k) gW[0][k] = sw[k] * inv_w;
        gb[0] = sb * inv_w;
      } else if constexpr (VARIANT == 4 || VARIANT == 5) {
        // 4: the rank's 21 values (20 weights + bias) travel as 21 consecutive LL words: ONE store
        //    instruction per peer (lanes 0..20) and ONE poll load per peer, redistributed through LDS;
        // 5: a single word per peer (the protocol's floor; the "gradient" is lane 0's value only)
        constexpr int NV = VARIANT == 4 ? 21 : 1;
        const int parity = (int)(seq & 1u);
        const uint64_t hi = (uint64_t)seq << 32;
        // the value lane l < NV contributes: weight l of chunk l / 5 (all lanes of a DPP row hold it), or the bias
        float* h = hand[seq & 1];
        if (i == 0) {
#pragma unroll
          for (int k = 0; k < KP; ++k) h[q * KP + k] = gW[0][k];
          if (q == 0) h[20] = gb[0];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const float mine = lane < NV ? h[lane] : 0.f;
        for (int p = 0; p < world; ++p) {
          if (p == rank || lane >= NV) continue;
          uint64_t PTDT_GLOBAL* dst = (uint64_t PTDT_GLOBAL*)(buf + p * region) + (int64_t)(parity * world + rank) * max_elems;
          __hip_atomic_store(dst + lane, hi | __float_as_uint(mine), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        float accv = 0.f;
        for (int p = 0; p < world; ++p) {  // rank order
          float val = mine;
          if (p != rank) {
            const uint64_t PTDT_GLOBAL* src = local + (int64_t)(parity * world + p) * max_elems + (lane < NV ? lane : 0);
            uint64_t w = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            for (uint32_t n = 0; __builtin_amdgcn_ballot_w64((uint32_t)(w >> 32) != seq) != 0 && n < (1u << 20); ++n)
              w = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            val = __uint_as_float((uint32_t)w);
          }
          accv += val;
        }
        h[64 + lane] = accv * inv_w;  // second half of the parity slot: the averaged values
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < KP; ++k) gW[0][k] = NV == 21 ? h[64 + q * KP + k] : h[64];
        gb[0] = NV == 21 ? h[64 + 20] : h[64];
      } else if constexpr (VARIANT == 3) {  // push (self included), then take the poller's sum
        if (i < world)
          lw::ll_push_chunk<KP, DOUT>(push_dst, rank, world, max_elems, seq, k0, DIN, true, q == 0, false, gW, gb);
        __builtin_amdgcn_s_barrier();
        const float* h = hand[seq & 1];
#pragma unroll
        for (int k = 0; k < KP; ++k) gW[0][k] = h[lane * (KP + 1) + k];
        gb[0] = h[lane * (KP + 1) + KP];
      } else {
        failed = __any(!ok);
#pragma unroll
        for (int k = 0; k < KP; ++k) gW[0][k] = lw::row16_sum(v[0][k]) * inv_w;
        gb[0] = lw::row16_sum(vb[0]) * inv_w;
      }
    }
#pragma unroll
    for (int k = 0; k < KP; ++k) W[k] = fmaf(-0.01f, gW[0][k], W[k]);
    x = fmaf(-0.01f, gb[0], x);
  }
  const long long t1 = (long long)__builtin_amdgcn_s_memtime();
  if (lane == 0) cycles[rank] = t1 - t0;
#pragma unroll
  for (int k = 0; k < KP; ++k) out[(rank * 64 + lane) * (KP + 1) + k] = W[k];
  out[(rank * 64 + lane) * (KP + 1) + KP] = x;
}

template <int V>
int run(uint64_t* buf, int world, int max_elems, int iters, int work, int* err, long long* cyc, float* out) {
  CK(hipMemset(buf, 0, (size_t)8 * world * 2 * world * max_elems));
  CK(hipMemset(err, 0, sizeof(int)));
  hipLaunchKernelGGL((k_exchange<V>), dim3(world), dim3(128), 0, 0, buf, world, max_elems, iters, work, err, cyc, out);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  int e = 0;
  std::vector<long long> c(world);
  std::vector<float> o((size_t)world * 64 * (KP + 1));
  CK(hipMemcpy(&e, err, sizeof(int), hipMemcpyDeviceToHost));
  CK(hipMemcpy(c.data(), cyc, sizeof(long long) * world, hipMemcpyDeviceToHost));
  CK(hipMemcpy(o.data(), out, o.size() * sizeof(float), hipMemcpyDeviceToHost));
  // rank-dependent data, identical initial weights: the weights stay bit-identical across ranks
  // only if every rank gets the same averaged gradient (the x column is rank-local and skipped)
  bool same = true;
  for (int r = 1; r < world; ++r)
    for (int l = 0; l < 64; ++l)
      same &= std::memcmp(&o[(size_t)l * (KP + 1)], &o[((size_t)r * 64 + l) * (KP + 1)], KP * sizeof(float)) == 0;
  long long mx = 0;
  for (long long v : c) mx = v > mx ? v : mx;
  std::printf("{\"variant\": %d, \"world\": %d, \"work\": %d, \"cycles_per_step\": %.1f, \"replicas_identical\": %s, "
              "\"err\": %d}\n",
              V, world, work, (double)mx / iters, same ? "true" : "false", e);
  return 0;
}

int main() {
  const int max_elems = 64, iters = 20000;
  uint64_t* buf;
  int* err;
  long long* cyc;
  float* out;
  CK(hipExtMallocWithFlags((void**)&buf, (size_t)8 * 8 * 2 * 8 * max_elems, hipDeviceMallocUncached));
  CK(hipMalloc(&err, sizeof(int)));
  CK(hipMalloc(&cyc, sizeof(long long) * 8));
  CK(hipMalloc(&out, sizeof(float) * 8 * 64 * (KP + 1)));
  for (int work : {0, 64}) {
    if (run<0>(buf, 1, max_elems, iters, work, err, cyc, out)) return 1;
    for (int world : {2, 4, 8}) {
      if (run<0>(buf, world, max_elems, iters, work, err, cyc, out)) return 1;
      if (run<1>(buf, world, max_elems, iters, work, err, cyc, out)) return 1;
      if (run<2>(buf, world, max_elems, iters, work, err, cyc, out)) return 1;
      if (run<3>(buf, world, max_elems, iters, work, err, cyc, out)) return 1;
      if (run<4>(buf, world, max_elems, iters, work, err, cyc, out)) return 1;
      if (run<5>(buf, world, max_elems, iters, work, err, cyc, out)) return 1;
      if (run<6>(buf, world, max_elems, iters, work, err, cyc, out)) return 1;
    }
  }
  return 0;
}
