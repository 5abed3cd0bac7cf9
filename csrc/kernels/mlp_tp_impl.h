// Persistent DDP step engine for Linear(Din,H)-ReLU-Linear(H,Dout) + loss + SGD,
// tensor-parallel across the waves of ONE workgroup, every product on MFMA.
// Shared by two translation units: mlp_tp.hip (exact fp32 operands, BF = false) and
// mlp_tp_bf16.hip (bf16 operands, BF = true; the bf16 section below).
//
// The toy MLP of BASELINE.json's north star (Linear(20,64)-ReLU-Linear(64,10),
// CE, SGD; per-device batch 32 as in ddp_gpus.py:34-39) is ~143K MACs per step:
// a latency problem, not a throughput one. Each of NW = H/16 waves owns 16 hidden
// units -- its rows of W1 (b1 folded in as input column Din against a constant-1
// input), the matching columns of W2, their momenta -- and runs its slice of the
// step with v_mfma_f32_16x16x4_f32 (exact fp32). Layouts are chosen so that every
// product's result is the next product's operand or lands on the weights it
// updates, lane for lane (D layout: lane (c = l&15, q = l>>4) holds [m = 4q+i][n = c]):
//
//   fwd1  HT[unit][row]  = W1aug . Xaug^T     A: w1r regs (unit c, input 4q+s), B: X rows (LDS)
//   fwd2  ZT_w[cls][row] = W2[:, slice] . HT  B = HT's result layout (K permuted to unit 4q+s)
//   ----  ONE workgroup barrier per step: the NW partial logits meet in LDS and
//         every wave sums them in wave order (identical bits in every wave)
//   loss  softmax / CE / MSE on the result layout (classes across lane groups:
//         permlane16/32 swaps; rows across the 16 lanes), in every wave
//   dH[row][unit] = dZ . W2[:, slice]         A = dZ's result layout, B = w2t regs
//   dW2[cls][unit] = dZ^T . H                 lands on w2t (W2[cls 4q+i][unit c])
//   dW1aug^T[in][unit] = Xaug^T . dH          B = dH's result layout; lands on w1r
//   SGD   in registers (padded inputs/classes have zero weights and gradients);
//         W2 is mirrored to a wave-private LDS tile in the forward's layout
//
// H^T and dZ^T go through wave-private LDS tiles for the two transposed operands
// of dW2 (no barrier: one wave's LDS ops complete in order). The next position's
// batch is staged into LDS by all threads during each step (loads issued at the
// top, written before the barrier; three slots), so operands are b128 LDS reads.
// Sampler lists live in LDS (three epoch slots); the entries of each future
// position are produced S+1 steps ahead of their use, C = min(8, S) positions at a
// time by all threads, so epoch transitions cost nothing. With an all-reduce (world > 1) every lane
// exchanges its gradient registers over xGMI with the LL protocol of
// comm/xgmi.h in a lane-major slot layout (tp_allreduce_lm: push to every peer,
// poll, sum in rank order: bit-identical replicas), then applies SGD.
//
// bf16 operands (BF, BASELINE.json config 2 "toy MLP bf16"): the same step with
// torch.autocast(bfloat16) semantics -- X, W1, b1, H, W2, b2, the logits, dZ, dH and every
// parameter gradient rounded to bf16 where autocast's bf16 Linear ops round them (fp32
// accumulation inside each product; softmax / CE in fp32 as autocast runs it), fp32 master
// weights and momentum with SGD in registers. Each product is ONE v_mfma_f32_16x16x32_bf16
// (K = 32 covers Din + bias <= 32, or the 32 batch rows) or v_mfma_f32_16x16x16_bf16 (K = the
// wave's 16 units or the <= 16 classes) per 16x16 tile instead of a chain of 4-8 dependent
// v_mfma_f32_16x16x4_f32. The K = 32 operands permute K the way the 16x16 result layout spreads a
// lane's 8 values over two 16-row tiles, so result registers feed the next product directly:
//   fwd1 (K = inputs): k = 8q + j <-> input 16 (j >> 2) + 4q + (j & 3)  (position tp_bpos): the
//        W1 master registers (W1[unit c][in 16 mt + 4q + i], dW1^T's result layout) ARE fwd1's A;
//   dW2 / dW1 (K = batch rows): k = 8q + j <-> row 16 (j & 1) + 4q + (j >> 1)  (position tp_rpos):
//        dH's result registers (rows 16 t + 4q + i) ARE dW1's B operand;
// and the LDS images (X rows, X^T, H^T, dZ^T) are staged in those orders, so every operand read
// from LDS is one 16-B read and every image write is one 8- or 4-B store (2-B for the transposes).
#pragma once
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "sampler.h"

namespace ptdt {
namespace {

constexpr int kTpThreadsMax = 320;  // up to 4 compute waves + the helper wave
#ifndef PTDT_TP_TWO_AHEAD  // helper wave: batch loads issued two positions ahead (a step of latency hidden)
#define PTDT_TP_TWO_AHEAD 1
#endif
constexpr bool kTpTwoAhead = PTDT_TP_TWO_AHEAD != 0;
#ifndef PTDT_TP_BF_POLL_PEERS
#define PTDT_TP_BF_POLL_PEERS 7
#endif
// bf16 engine, float4-staged class-index CE instances (the toy): peers polled per round (packed words;
// 7 = W = 8 in one round); the others use 4 (7 spilled 28-46 VGPRs there)
constexpr int kTpBfPollPeers = PTDT_TP_BF_POLL_PEERS;
using f4 = __attribute__((ext_vector_type(4))) float;
using f2 = __attribute__((ext_vector_type(2))) float;
using bf8 = __attribute__((ext_vector_type(8))) __bf16;   // 16x16x32 bf16 operand (8 K values per lane)
using s4 = __attribute__((ext_vector_type(4))) short;     // 16x16x16 bf16 operand (4 K values per lane)
using s8 = __attribute__((ext_vector_type(8))) short;
using u2v = __attribute__((ext_vector_type(2))) unsigned int;
using u4v = __attribute__((ext_vector_type(4))) unsigned int;

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
__device__ __forceinline__ f4 mfma_k32(bf8 a, bf8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }
__device__ __forceinline__ f4 mfma_k16(s4 a, s4 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0); }
// round to bf16 precision, kept as f32 (v_cvt_pk_bf16_f32 + shift)
__device__ __forceinline__ float bfr(float x) { return bf16_to_f32(f32_to_bf16(x)); }
__device__ __forceinline__ s4 pack_bf4(float a, float b, float c, float d) {
  return __builtin_bit_cast(s4, u2v{pack_bf16x2(a, b), pack_bf16x2(c, d)});
}
__device__ __forceinline__ bf8 pack_bf8(const float (&v)[8]) {
  return __builtin_bit_cast(bf8, u4v{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                                     pack_bf16x2(v[6], v[7])});
}
// positions of input x / batch row x (< 32) in the K = 32 operand images (see the header)
__host__ __device__ __forceinline__ int tp_bpos(int x) { return 8 * ((x & 15) >> 2) + (x & 3) + 4 * (x >> 4); }
__host__ __device__ __forceinline__ int tp_rpos(int x) { return 2 * (x & 15) + (x >> 4); }
constexpr unsigned short kBf16One = 0x3F80;

// Wait states between the end of an MFMA chain and the first VALU read of its result,
// padded explicitly: with a (uniform) branch between the last v_mfma_f32_16x16x4_f32
// and the read, hipcc's hazard recognizer padded only for the fall-through path
// (s_nop 1 before reading the 4th result register on the taken one), and the read
// returned a stale value (the 4th register of the dW1^T tile, only when no other MFMA
// chain followed). 8-pass XDL -> VALU read needs 11; scheduling is fenced on both sides.
__device__ __forceinline__ void mfma_settle() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 4" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// across the 4 lane groups (DPP rows) of a column: permlane16 then permlane32
// swaps, symmetric pairing -> every lane gets the same bits
__device__ __forceinline__ float rows4_sum(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  v = __int_as_float(p[0]) + __int_as_float(p[1]);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(q[0]) + __int_as_float(q[1]);
}
__device__ __forceinline__ float rows4_max(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  v = fmaxf(__int_as_float(p[0]), __int_as_float(p[1]));
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return fmaxf(__int_as_float(q[0]), __int_as_float(q[1]));
}

struct TpDims {
  int B, Din, H, Dout, NW, estride;
  int oW1, ob1, oW2, ob2, np;
};

__device__ __forceinline__ TpDims tp_dims(const FusedMlpArgs& a, const PersistArgs& pa) {
  TpDims d;
  d.B = a.B; d.Din = a.Din; d.H = a.H; d.Dout = a.Dout;
  d.NW = a.H / 16;
  d.estride = al4(pa.num_samples);
  const int hb = a.has_bias != 0;
  d.oW1 = 0;
  d.ob1 = a.H * a.Din;
  d.oW2 = d.ob1 + (hb ? a.H : 0);
  d.ob2 = d.oW2 + a.Dout * a.H;
  d.np = d.ob2 + (hb ? a.Dout : 0);
  return d;
}

__device__ __forceinline__ float sgd1(float& w, float& m, float g, bool first, float lr, float mu, float damp, float wd,
                                      int nesterov, bool mom) {
  float d = fmaf(wd, w, g);
  if (mom) {
    const float buf = first ? d : fmaf(mu, m, (1.f - damp) * d);
    m = buf;
    d = nesterov ? fmaf(mu, buf, d) : buf;
  }
  w = fmaf(-lr, d, w);
  return w;
}

// Lane-major gradient all-reduce (replaces tp_allreduce on the step's critical path).
// Every rank runs the same lane -> parameter mapping, so the exchange need not use the
// flat parameter index: value k of wave w, lane l travels in LL slot (w NV + k) 64 + l.
// One push instruction then writes 64 consecutive words (512 contiguous bytes, 4 cache
// lines) instead of 64 words strided by Din (64 separate uncached transactions), and one
// poll instruction reads them back the same way -- round 2's flat-index pushes were
// 3.3K scattered uncached writes per step (share-GPU W=2: 6.4 us/step vs 2.8 at W=1).
// Polls of G peers are in flight together (G = 3 for the index-CE / vector-staging instances, whose registers allow
// it: the W - 1 other ranks in ceil((W - 1) / G) poll rounds, W = 4 in one and W = 8 in 3 -- 2 for the
// others); the loop is uniform (ballot exit,
// every lane re-polls its whole set), contributions are summed in rank order (own value
// from the register): bit-identical replicas. Padded values (zero gradients) travel too.
// PK (the bf16 engine, whose gradients are bf16 values by autocast semantics): two values per LL
// word -- (NV + 1) / 2 words per lane instead of NV, half the pushes, polls and poll registers, so
// more peers' polls fit in flight at once (G). The sum is the same fp32 rank-ordered one.
template <int NV, int G, bool PK = false>
__device__ __forceinline__ bool tp_allreduce_lm(const XgmiArgs& x, uint32_t seq, float (&v)[NV], int wave, int lane) {
  constexpr int NW = PK ? (NV + 1) / 2 : NV;  // LL words per lane
  const int parity = (int)(seq & 1u);
  const uint64_t hi = (uint64_t)seq << 32;
  const bool drop = x.drop_push != 0u && seq >= x.drop_push;
  const int base = wave * NW * 64 + lane;
  uint32_t pay[NW];
#pragma unroll
  for (int k = 0; k < NW; ++k) {
    if constexpr (PK)
      pay[k] = (__float_as_uint(v[2 * k]) >> 16) | (2 * k + 1 < NV ? __float_as_uint(v[2 * k + 1]) & 0xffff0000u : 0u);
    else
      pay[k] = __float_as_uint(v[k]);
  }
  for (int p = 0; p < x.world; ++p) {
    if (p == x.rank || drop) continue;
    uint64_t PTDT_GLOBAL* const dst =
        (uint64_t PTDT_GLOBAL*)x.peers[p] + (int64_t)(parity * x.world + x.rank) * x.max_elems + base;
#pragma unroll
    for (int k = 0; k < NW; ++k)
      __hip_atomic_store(dst + k * 64, hi | (uint64_t)pay[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  float acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = 0.f;
  bool ok = true;
  bool own = false;  // this rank's value added (rank order: just before the first higher peer)
  const int np = x.world - 1;  // the OTHER ranks, polled in groups of G in increasing rank order
  auto peer = [&](int i) { return i < x.rank ? i : i + 1; };
  for (int i0 = 0; i0 < np; i0 += G) {
    uint64_t w[G][NW];
    auto issue = [&]() {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const bool real = i0 + g < np;  // uniform
        const uint64_t PTDT_GLOBAL* src =
            (const uint64_t PTDT_GLOBAL*)x.local + (int64_t)(parity * x.world + (real ? peer(i0 + g) : 0)) * x.max_elems + base;
#pragma unroll
        for (int k = 0; k < NW; ++k)
          w[g][k] = real ? __hip_atomic_load(src + k * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : hi;
      }
    };
    issue();
    for (uint32_t polls = 0;; ++polls) {
      bool m = false;
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int k = 0; k < NW; ++k) m |= (uint32_t)(w[g][k] >> 32) != seq;
      if (__builtin_amdgcn_ballot_w64(m) == 0) break;
      if (polls >= x.max_polls) {
        __hip_atomic_store(x.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ok = false;
        break;
      }
      issue();
    }
    if (!ok) break;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (i0 + g >= np) break;
      if (!own && peer(i0 + g) > x.rank) {
#pragma unroll
        for (int k = 0; k < NV; ++k) acc[k] += v[k];
        own = true;
      }
#pragma unroll
      for (int k = 0; k < NW; ++k) {
        const uint32_t u = (uint32_t)w[g][k];
        if constexpr (PK) {
          acc[2 * k] += __uint_as_float(u << 16);
          if (2 * k + 1 < NV) acc[2 * k + 1] += __uint_as_float(u & 0xffff0000u);
        } else {
          acc[k] += __uint_as_float(u);
        }
      }
    }
  }
  if (!own)
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] += v[k];
  const float inv = 1.f / (float)x.world;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = acc[k] * inv;
  return ok;
}

// LDS floats of one staged batch slot: X rows [32][ldx], X^T [16 MT][ldxt], targets [32][16]
template <int MT>
struct TpStage {
  static constexpr int LDX = 16 * MT + 4;  // b128 reads of 4 consecutive inputs
  static constexpr int LDXT = 36;          // b128 reads of 4 consecutive rows
  static constexpr int XT_OFF = 32 * LDX;
  static constexpr int Y_OFF = XT_OFF + 16 * MT * LDXT;
  static constexpr int FLOATS = Y_OFF + 32 * 16;
};
// bf16 operand images (BF): X rows [32][kTpLB] (inputs at tp_bpos), X^T [32 inputs][kTpLB] (rows at
// tp_bpos), both bf16 (offsets in floats), targets [32][16] f32 as above
constexpr int kTpLB = 40;  // bf16 per row of a K = 32 image: 64 B of data + 16 B pad (80-B rows, 16-B aligned)
struct TpStageB {
  static constexpr int LDX = kTpLB;
  static constexpr int XT_OFF = 32 * kTpLB / 2;
  static constexpr int Y_OFF = XT_OFF + 32 * kTpLB / 2;
  static constexpr int FLOATS = Y_OFF + 32 * 16;
};
constexpr int kTpLDZB = 20;  // bf16 per row of the row-major dZ image (BF): 8-B reads of 4 classes
constexpr int kTpLD2 = 20;  // W2 slice (classes x 16 units), b128 rows
constexpr int kTpLDT = 36;  // per-wave transposes: 16 (class / unit) x 32 rows
constexpr int kTpLDZ = 20;  // shared dZ, row-major: 32 rows x 16 classes, b128 rows
constexpr int kTpLossRing = 32;  // loss-ring slots (power of two)
constexpr int kTpLossFlush = 16; // steps per flush: the slots being added are never the one written meanwhile
__host__ __device__ __forceinline__ int tp_wave_floats() { return 16 * kTpLD2 + 2 * 16 * kTpLDT + 16; }
__host__ __device__ __forceinline__ int tp_stage_floats(int MT, bool bf) {
  return bf ? TpStageB::FLOATS : 32 * (16 * MT + 4) + 16 * MT * 36 + 32 * 16;
}

// MT: 16-input tiles of the augmented input (Din inputs + a constant-1 column carrying b1);
// VX: X rows staged as float4 chunks (Din and the row stride multiples of 4, X 16-B aligned);
// ST: phase timers compiled in (diagnostic build: uniform branches around s_memtime)
// LDS position of input `in` in a staged X row: the two 2-bit fields of the input's index inside
// its 16-input tile are swapped, so the b128 read at 16 mt + 4 q hands lane group q the inputs
// 16 mt + 4 s + q (s = 0..3) -- fwd1's K-step s then covers 4 CONSECUTIVE inputs, and the K-steps
// of the last tile that hold only padding (inputs >= Din + bias) can be skipped (KL)
__host__ __device__ __forceinline__ int tp_xpos(int in) { return (in & ~15) + 4 * (in & 3) + ((in >> 2) & 3); }

// BF: bf16 operands (header); MT then counts dW1's 16-input result tiles (fwd1 is one K = 32 MFMA)
template <int MT, int LOSS, bool AR, bool VX, bool ST, int KL = 4, bool BF = false>
__global__ void __launch_bounds__(kTpThreadsMax) mlp_tp_kernel(FusedMlpArgs a, PersistArgs pa) {
  // No implicit FMA contraction: the compiler may contract differently in a peeled
  // first iteration than in the loop body, which made a run split into several
  // launches differ in the last bit from one long launch. Fused ops are explicit
  // (fmaf in sgd1, MFMA).
#pragma clang fp contract(off)
  using St = typename std::conditional<BF, TpStageB, TpStage<MT>>::type;
  constexpr int LDX = St::LDX, LD2 = kTpLD2, LDT = kTpLDT;
  constexpr int LDXT = BF ? kTpLB : TpStage<MT>::LDXT;
  extern __shared__ float lds[];
  // the pointers the prologue dereferences, loaded in one batch with the dimensions (pinned): left to
  // the compiler, four dependent kernel-argument loads led the prologue (see linear_wave_impl.h)
  {
    const float* const x_arg = a.X;
    const int64_t* const yi_arg = a.Yi;
    const float* const p_arg = a.P;
    const int32_t* const idx_arg = pa.idx;
    const float* const losses_arg = pa.losses;
    const int32_t* const lcache_arg = pa.lcache;
    const int ns_arg = pa.num_samples, b_arg = a.B, din_arg = a.Din, h_arg = a.H;
    asm volatile("" ::"s"(x_arg), "s"(yi_arg), "s"(p_arg), "s"(idx_arg), "s"(losses_arg), "s"(lcache_arg), "s"(ns_arg),
                 "s"(b_arg), "s"(din_arg), "s"(h_arg));
  }
  const TpDims d = tp_dims(a, pa);
  // diagnostic (ST): kernel entry and three prologue marks (10 ns ticks; waits forced at each mark)
  const int64_t r_entry = ST ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
  int64_t r_pro[6] = {0, 0, 0, 0, 0, 0};
  auto pstamp = [&](int k) {
    if constexpr (ST) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      r_pro[k] = (int64_t)__builtin_amdgcn_s_memrealtime();
    }
  };
  const int tid = (int)threadIdx.x;
  const int T = (int)blockDim.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l = tid & 63, c = l & 15, q = l >> 4;
  const int B = d.B, Din = d.Din, H = d.H, Dout = d.Dout, NW = d.NW;
  const bool hb = a.has_bias != 0;
  const bool use_mom = a.mom != nullptr && a.momentum != 0.f;
  const float lr = a.lr, mu = a.momentum, damp = a.dampening, wd = a.weight_decay;
  const bool plain_sgd = !use_mom && wd == 0.f;
  const int nesterov = a.nesterov;

  // ---- LDS carve-up
  // [3][estride] epoch lists: a producer one epoch ahead never overwrites a list a
  // lagging wave may still read (position P's and P+1's epochs)
  int* const elist = reinterpret_cast<int*>(lds);
  float* const stage0 = lds + 3 * d.estride;                 // [3] staged batches (TpStage)
  float* const xbuf = stage0 + 3 * St::FLOATS;               // [2][NW][2 tiles][64 lanes][4] partial logits
  float* const wbase = xbuf + 2 * NW * 64 * 8 + tp_wave_floats() * w;
  // Feistel keys of epochs e (slot e & 3, 12 ints: key[4], maskL, maskR, hb, n, epoch), after the wave regions
  int* const fkeys = reinterpret_cast<int*>(xbuf + 2 * NW * 64 * 8 + tp_wave_floats() * NW);
  float* const W2m = wbase;                                   // [16 classes][LD2] W2[:, slice] (fwd layout)
  float* const Th = W2m + 16 * LD2;                           // [16 units][LDT] H^T of this slice
  float* const Tdz = Th + 16 * LDT;                           // [16 classes][LDT] dZ^T
  float* const B2m = Tdz + 16 * LDT;                          // [16] b2 (the forward's class-4q+i reads)
  // [kTpLossRing][64] loss ring (16-B aligned, after the keys): wave 0 stores each lane's
  // scaled loss share per step; every kTpLossFlush steps all waves add the shares of the
  // past kTpLossFlush slots in lane order
  float* const lring = lds + al4((int)(reinterpret_cast<float*>(fkeys) - lds) + 48);
  // shared dZ of the step (written by the row slices' owners before the second barrier):
  // row-major [32][kTpLDZ] and transposed [16 classes][LDT] with interleaved tiles
  float* const dZr = lring + kTpLossRing * 64;
  float* const dZt = dZr + 32 * kTpLDZ;
  auto flush_losses = [&](int lo, int hi) {  // steps [lo, hi), hi - lo <= kTpLossFlush (helper wave)
    const int j = l;
    if (j < hi - lo) {
      const int step = lo + j;
      const f4* sh = reinterpret_cast<const f4*>(lring + (step & (kTpLossRing - 1)) * 64);
      float acc = 0.f;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const f4 v = sh[u];
        acc += v[0];
        acc += v[1];
        acc += v[2];
        acc += v[3];
      }
      pa.losses[step] = acc;
    }
  };
  auto list = [&](int e) { return elist + (e % 3) * d.estride; };
  auto stage = [&](int slot) { return stage0 + slot * St::FLOATS; };

  // ---- resident state of the compute waves, loaded first so that its latency hides under the
  // sampler lists and the staging below (hipcc also spills less this way: 0-41 vs 1-46 VGPRs): this wave's W1 rows (b1 as column Din) and W2 columns in
  // MFMA result layouts, so the gradients land on them lane for lane and SGD runs in registers:
  //   w1r[mt][i] = W1aug[unit 16w + c][input 16 mt + 4q + i]   (= dW1^T's layout)
  //   w2t[i]     = W2[class 4q + i][unit 16w + c]              (= dW2's layout)
  //   b2c        = b2[class c] (= db2's layout: the column sums of dZ^T)
  const int unit = 16 * w + c;
  float w1r[MT][4], m1r[MT][4], w2t[4], m2t[4], b2c = 0.f, mb2c = 0.f;
  int opt_step = 0;
  uint32_t seq = 0u;
  bool failed = false;
  auto load_state = [&]() {
    const auto P = gptr(a.P);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // fp32: fwd1's K-step i of tile mt, lane group q; BF: dW1^T's result row 4q + i of tile mt
        const int in = BF ? 16 * mt + 4 * q + i : 16 * mt + 4 * i + q;
        const int off = in < Din ? d.oW1 + unit * Din + in : (hb && in == Din ? d.ob1 + unit : -1);
        w1r[mt][i] = off >= 0 ? P[off] : 0.f;
        m1r[mt][i] = (off >= 0 && use_mom) ? a.mom[off] : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cls = 4 * q + i;
      const bool real = cls < Dout;
      w2t[i] = real ? P[d.oW2 + cls * H + unit] : 0.f;
      m2t[i] = (real && use_mom) ? a.mom[d.oW2 + cls * H + unit] : 0.f;
    }
    b2c = (hb && c < Dout) ? P[d.ob2 + c] : 0.f;
    mb2c = (hb && c < Dout && use_mom) ? a.mom[d.ob2 + c] : 0.f;
    opt_step = a.opt_step ? *a.opt_step : 0;
    seq = AR ? *a.ar.seq : 0u;
    failed = AR && *a.ar.err != 0;
  };
  if (w < NW) load_state();
  pstamp(0);  // resident state loaded

  // ---- sampler lists: epoch e0 whole, epoch e0+1 up to batch j0 (entries of later
  // positions are produced S+1 steps ahead inside the loop)
  const int ns = pa.num_samples;
  const int S = (ns + B - 1) / B;
  // the start position: from the arguments (launch_at), or the device cursor only on the plain-launch
  // path -- written as a value select, the compiler loaded it through a flat load of a pointer
  // selected between the two (a dependent memory round trip on every launch; see linear_wave_impl.h)
  const int has_start = pa.has_start, start_e = pa.start_e, start_j = pa.start_j;
  asm volatile("" ::"s"(has_start), "s"(start_e), "s"(start_j));
  int e0 = start_e, j0 = start_j;
  if (!has_start) {
    e0 = pa.cursor[0];
    j0 = pa.cursor[1];
  }
  const int n = pa.n_steps;
  const uint32_t Nn = (uint32_t)pa.N;
  const ListCache lc{pa.lcache, pa.ltag, d.estride};
  // rank position of list entry i: (rank + W i) mod N without a 64-bit remainder
  auto rank_pos = [&](int i) {
    uint32_t pos = (uint32_t)pa.rank + (uint32_t)pa.W * (uint32_t)i;
    while (pos >= Nn) pos -= Nn;
    return pos;
  };
  // epochs e0 and e0+1 whole, from the launch-to-launch cache when it holds them (both slots' loads
  // in flight together). Epoch e0+1's entries of positions before j0 are never produced by the
  // helper (later ones are, with the same values): a launch that resumes where the last one stopped
  // loads both lists instead of running the Feistel permutation for up to a whole epoch on the way
  // to step 0 (round 4: ~1.8 us of the prologue)
  rank_epoch_indices_or2(given_list(pa, e0), list(e0), given_list(pa, e0 + 1), list(e0 + 1), Nn, pa.W, pa.rank, ns,
                         pa.seed, e0, pa.shuffle, tid, T, lc);
  pstamp(1);  // epochs e0 and e0+1 in LDS
  // Feistel keys of the epochs the producer will need (computed by one thread, one
  // epoch ahead of use: a produce call reads te, te + 1 and prepares te + 2)
  const bool feistel = pa.idx == nullptr && pa.shuffle;
  auto keys_store = [&](int e) {
    int* const k = fkeys + (e & 3) * 12;
    FeistelPerm fp;
    fp.init(pa.seed, e, Nn);
#pragma unroll
    for (int r = 0; r < 4; ++r) k[r] = (int)fp.key[r];
    k[4] = (int)fp.maskL;
    k[5] = (int)fp.maskR;
    k[6] = fp.hb;
    k[7] = (int)fp.n;
    k[8] = e;
  };
  auto keys_load = [&](int e) {
    const int* const k = fkeys + (e & 3) * 12;
    FeistelPerm fp;
#pragma unroll
    for (int r = 0; r < 4; ++r) fp.key[r] = (uint32_t)k[r];
    fp.maskL = (uint32_t)k[4];
    fp.maskR = (uint32_t)k[5];
    fp.hb = k[6];
    fp.n = (uint32_t)k[7];
    return fp;
  };
  pstamp(2);  // epoch e0+1's list up to the cursor (the Feistel keys follow the next barrier)
  // staged batch slots: zeros, and the constant-1 input column (b1 rides in W1's
  // column Din) in X and X^T; the per-step writes only touch columns < Din
  // (16-B zero stores, then the constant-1 entries after a barrier: the per-element index
  // arithmetic of a one-pass fill cost ~1-2 us of every launch's prologue)
  static_assert(St::FLOATS % 4 == 0, "float4 fill");
  for (int e = tid; e < 3 * St::FLOATS / 4; e += T) reinterpret_cast<f4*>(stage0)[e] = f4{0.f, 0.f, 0.f, 0.f};
  // loss ring: each step writes its 32 row losses into entries 0..31 of its slot; 32..63 stay 0
  for (int e = tid; e < kTpLossRing * 64; e += T) lring[e] = 0.f;
  __syncthreads();
  if (hb) {
    for (int e = tid; e < 3 * 64; e += T) {  // per slot: X[row][Din] and X^T[Din][row], rows 0..31
      float* const st = stage0 + (e >> 6) * St::FLOATS;
      const int r = e & 31;
      if constexpr (BF) {
        unsigned short* const sb = reinterpret_cast<unsigned short*>(st);
        if ((e & 63) < 32) sb[r * LDX + tp_bpos(Din)] = kBf16One;
        else sb[2 * St::XT_OFF + Din * LDXT + tp_rpos(r)] = kBf16One;
      } else {
        if ((e & 63) < 32) st[r * LDX + tp_xpos(Din)] = 1.f;
        else st[St::XT_OFF + Din * LDXT + r] = 1.f;
      }
    }
  }
  pstamp(3);  // lists, staging-slot init (and the compute waves' state loads) done
  __syncthreads();
  pstamp(4);
  // Feistel keys of epochs e0+1 .. e0+3 (read only by the helper wave, after barrier 1 of step 0):
  // lanes 0-2 of wave 0 while the helper stages step 0 below, where the compute waves only wait (before
  // the first barrier they were ~0.5 us of every launch's prologue). Lane 3 invalidates the fourth slot,
  // whose tag is LDS left over from an earlier kernel on this CU: a stale tag equal to a later epoch made
  // the producer skip that epoch's keys and cycle-walk another launch's permutation (sample count
  // N' != N: the walk from an input >= 2^bits' never ends).
  if (feistel && w == 0 && l < 4) {
    if (l < 3) keys_store(e0 + 1 + l);
    else fkeys[(e0 & 3) * 12 + 8] = -0x7fffffff - 1;
  }
  if (tid == 0 && pa.idx == nullptr) {
    list_cache_publish(lc, e0);
    list_cache_publish(lc, e0 + 1);
  }

  // Helper wave (w == NW): owns the sampler lists and the batch staging, so the NW compute
  // waves run only the step's math. It meets the compute waves at their two barriers per step and
  // splits its work between the two phases they leave it:
  //   * before barrier 1 (the compute waves' backward + SGD + forward): stage position k+1 into slot
  //     (k+1) % 3 (rows and X^T; float4 instances write the rows loaded during step k-1 and put
  //     position k+2's loads in flight) -- the slot was last read in step k-2's backward (before
  //     barrier 1 of k-1) and is next read in step k+1 (after barrier 2 of k);
  //   * between the barriers (the compute waves' loss rows): produce ONE list position, S+2 ahead
  //     of the step (cycle-walking Feistel of the device sampler; the Feistel keys stay in
  //     registers within an epoch; three LDS epoch slots keep it clear of the ones still read),
  //     and every 16 steps add the loss shares wave 0 left in the LDS ring.
  // Round 5 produced 8 positions every 8 steps before barrier 1 (a runtime division per entry, a
  // per-lane choice between two key structs, the keys reloaded every call): ~4.6K cycles per call,
  // and with the staging on a SIMD shared with a compute wave the helper reached barrier 1 ~500
  // cycles after the compute waves in every step (profiles/r6_tp_bf16.md, helper phase stamps).
  // Round 2 ran all of this on the compute waves (~900 of ~7500 cycles per step).
  FeistelPerm fcur;  // keys of epoch pe (the position produced next: (pe, pj))
  auto keys_for = [&](int e) {  // the keys of epoch e in fcur (stored first when its slot holds another)
    if (l == 0 && fkeys[(e & 3) * 12 + 8] != e) keys_store(e);
    fcur = keys_load(e);
  };
  auto produce_one = [&](int pe, int pj) {  // lane = row of position (pe, pj); B <= 32
    const int i = pj * B + l;
    if (l < B && i < ns) {
      int v;
      if (pa.idx != nullptr) v = given_list(pa, pe)[i];
      else if (feistel) v = (int)fcur(rank_pos(i));
      else v = (int)rank_pos(i);
      list(pe)[i] = v;
    }
  };

  // ---- batch staging (helper lanes l = 0..63): item e = l + 64 k of the 32-row tile (float4
  // chunks when VX, else single floats) for k below a count uniform over the wave; the last
  // item is repeated past the end (identical writes), rows past the batch read clamped rows.
  constexpr int KX = VX ? 4 : 16, KY = 8;
  const auto X = gptr(a.X);
  const int ldx = a.ldx > 0 ? a.ldx : Din;
  const int xper = VX ? Din / 4 : Din;  // items per row
  const int nkx = (32 * xper + 63) / 64;
  int xrow[KX], xcol[KX];
#pragma unroll
  for (int k = 0; k < KX; ++k) {
    const int e = min(l + k * 64, 32 * xper - 1);
    xrow[k] = e / xper;
    xcol[k] = e - xrow[k] * xper;
  }
  constexpr bool YI = LOSS == kLossCEIndex;
  const int yper = YI ? 1 : Dout;
  const int nky = (32 * yper + 63) / 64;
  int yrow[KY], ycol[KY];
#pragma unroll
  for (int k = 0; k < KY; ++k) {
    const int e = min(l + k * 64, 32 * yper - 1);
    yrow[k] = e / yper;
    ycol[k] = e - yrow[k] * yper;
  }
  using XV = typename std::conditional<VX, f4, float>::type;  // a float4 chunk or one float
  XV xv[KX];
  float yv[KY];
  int xsel[KX], ysel[KY];
  auto stage_sel = [&](int E, int J) {
    const int nb = min(B, ns - J * B);
    const int* const li = list(E) + J * B;
#pragma unroll
    for (int k = 0; k < KX; ++k)
      if (k < nkx) xsel[k] = li[min(xrow[k], nb - 1)];
#pragma unroll
    for (int k = 0; k < KY; ++k)
      if (k < nky) ysel[k] = li[min(yrow[k], nb - 1)];
  };
  auto stage_issue = [&]() {
#pragma unroll
    for (int k = 0; k < KX; ++k) {
      if (k < nkx) {
        if constexpr (VX) {
          xv[k] = *reinterpret_cast<const f4*>(a.X + (int64_t)xsel[k] * ldx + 4 * xcol[k]);
        } else {
          xv[k] = X[(int64_t)xsel[k] * ldx + xcol[k]];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < KY; ++k) {
      if (k < nky) {
        // the low dword of the int64 label only (a dwordx2 load's dead high half was reused
        // as a temporary behind a vmcnt(0))
        if constexpr (YI) yv[k] = __int_as_float(reinterpret_cast<const int*>(a.Yi)[2 * (int64_t)ysel[k]]);
        else yv[k] = gptr(a.Yf)[(int64_t)ysel[k] * Dout + ycol[k]];
      }
    }
  };
  auto stage_write = [&](int slot) {
    float* const st = stage(slot);
#pragma unroll
    for (int k = 0; k < KX; ++k) {
      if (k < nkx) {
        const int row = xrow[k];
        if constexpr (BF) {
          // bf16 images: inputs 4 xcol .. 4 xcol + 3 sit at 4 consecutive positions of the row
          // (tp_bpos keeps aligned groups of 4 together): one 8-B store; X^T: one 2-B store each
          unsigned short* const sb = reinterpret_cast<unsigned short*>(st);
          if constexpr (VX) {
            *reinterpret_cast<u2v*>(sb + row * LDX + tp_bpos(4 * xcol[k])) =
                u2v{pack_bf16x2(xv[k][0], xv[k][1]), pack_bf16x2(xv[k][2], xv[k][3])};
#pragma unroll
            for (int i = 0; i < 4; ++i)
              sb[2 * St::XT_OFF + (4 * xcol[k] + i) * LDXT + tp_rpos(row)] = f32_to_bf16(xv[k][i]);
          } else {
            const unsigned short v16 = f32_to_bf16(xv[k]);
            sb[row * LDX + tp_bpos(xcol[k])] = v16;
            sb[2 * St::XT_OFF + xcol[k] * LDXT + tp_rpos(row)] = v16;
          }
        } else if constexpr (VX) {
          // inputs 4 xcol + i land at positions (4 xcol & ~15) + 4 i + (xcol & 3) (tp_xpos)
          float* const xr = st + row * LDX + ((4 * xcol[k]) & ~15) + (xcol[k] & 3);
#pragma unroll
          for (int i = 0; i < 4; ++i) xr[4 * i] = xv[k][i];
#pragma unroll
          for (int i = 0; i < 4; ++i) st[St::XT_OFF + (4 * xcol[k] + i) * LDXT + row] = xv[k][i];
        } else {
          st[row * LDX + tp_xpos(xcol[k])] = xv[k];
          st[St::XT_OFF + xcol[k] * LDXT + row] = xv[k];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < KY; ++k)
      if (k < nky) st[St::Y_OFF + (YI ? yrow[k] : yrow[k] * 16 + ycol[k])] = yv[k];
  };
  // position of step 0 staged synchronously (helper), visible to all after the barrier; with
  // two-ahead staging, position 1's loads are then left in flight (the loop's step 0 writes them).
  // Float4 staging only: the scalar form's 16 staged items per lane stay live across the step and
  // spilled 12 VGPRs.
  constexpr bool TA = kTpTwoAhead && VX;
  if (w == NW) {
    stage_sel(e0, j0);
    stage_issue();
    stage_write(0);
    if constexpr (TA) {
      const bool w0 = j0 + 1 == S;
      stage_sel(w0 ? e0 + 1 : e0, w0 ? 0 : j0 + 1);
      stage_issue();
    }
  }
  __syncthreads();
  pstamp(5);  // step 0's batch staged: the loop starts

  const float inv_full = 1.f / (float)(LOSS == kLossMSE ? B * Dout : B);
  const int ce0 = e0, cj0 = j0;
  if (w == NW) {
    // ================================================================ helper wave
    int ce = ce0, cj = cj0, sc = 0;
    // (ST) [0] rest of the step's work [1] barrier-1 wait [2] barrier-2 wait [3] produce [4] stage_write
    // [5] stage_sel + issue [6] loss flush
    int64_t h_acc[7] = {0, 0, 0, 0, 0, 0, 0}, h_mark = ST ? (int64_t)__builtin_amdgcn_s_memtime() : 0;
    auto h_tick = [&](int ph) {
      if constexpr (ST) {
        const int64_t t = (int64_t)__builtin_amdgcn_s_memtime();
        h_acc[ph] += t - h_mark;
        h_mark = t;
      }
    };
    // list positions produced: (e0, j0) + S + 1 here, then (e0, j0) + S + 2 + k in step k -- every
    // position past the prologue's two epochs exactly once, each >= 1 step before it is staged
    int pe = cj0 + 1 == S ? ce0 + 2 : ce0 + 1, pj = cj0 + 1 == S ? 0 : cj0 + 1;
    auto advance = [&]() {
      if (++pj == S) {
        pj = 0;
        ++pe;
        if (feistel) keys_for(pe);
      }
    };
    if (feistel) keys_for(pe);
    produce_one(pe, pj);
    advance();
    for (int k = 0; k < n; ++k) {
      const bool wrap = cj + 1 == S;
      const int ne = wrap ? ce + 1 : ce, nj = wrap ? 0 : cj + 1;
      const int sn = sc == 2 ? 0 : sc + 1;
      h_tick(0);
      if constexpr (TA) {
        // position k + 1 was loaded during step k - 1 (a whole step of latency hidden): write it, then
        // put position k + 2's loads in flight across this step's barriers (stale-but-valid past the
        // launch: its entries were produced at least one step ago)
        stage_write(sn);
        h_tick(4);
        const bool wrap2 = nj + 1 == S;
        stage_sel(wrap2 ? ne + 1 : ne, wrap2 ? 0 : nj + 1);
        stage_issue();
        h_tick(5);
      } else {
        stage_sel(ne, nj);  // position k + 1 (stale-but-valid past the launch)
        stage_issue();
        h_tick(5);
        stage_write(sn);
        h_tick(4);
      }
      __syncthreads();  // barrier 1 of step k (partial logits)
      h_tick(1);
      produce_one(pe, pj);
      advance();
      h_tick(3);
      // shares of steps [k-16, k): written by wave 0 before barrier 1 of step k - 1 or earlier
      if (k > 0 && (k & (kTpLossFlush - 1)) == 0) flush_losses(k - kTpLossFlush, k);
      h_tick(6);
      __syncthreads();  // barrier 2 of step k (dZ slices)
      h_tick(2);
      ce = ne;
      cj = nj;
      sc = sn;
    }
    if (ST && l == 0 && pa.stamps_n >= 30)  // the helper's own split (h_acc above)
      for (int q2 = 0; q2 < 7; ++q2) pa.stamps[23 + q2] += h_acc[q2];
    if (n > 0) {  // the remaining loss shares (every step's share written before the final barrier)
      __syncthreads();
      const int kf = ((n - 1) / kTpLossFlush) * kTpLossFlush;  // the loop flushed [0, kf)
      for (int lo = kf; lo < n; lo += kTpLossFlush) flush_losses(lo, min(n, lo + kTpLossFlush));
    }
    return;
  }

  // ================================================================ compute waves
  // (resident state loaded at the top of the kernel; its forward-layout LDS mirrors now)
  // BF: bf16 operand copies of the resident weights -- fwd1's A (W1aug[unit c][in tp_bpos^-1(8q + j)]
  // = w1r[j >> 2][j & 3]) and dH's B (W2[class 4q + j][unit c] = w2t[j]) -- and a bf16 forward
  // mirror of W2 (fwd2's A: W2[class c][unit 4q + j], 8-B reads); b2's mirror holds bf16(b2)
  bf8 w1b;
  s4 w2b;
  unsigned short* const W2mb = reinterpret_cast<unsigned short*>(W2m);
  auto mirror = [&]() {
    if constexpr (BF) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (j >> 2) < MT ? w1r[(j >> 2) < MT ? (j >> 2) : 0][j & 3] : 0.f;
      w1b = pack_bf8(v);
      w2b = pack_bf4(w2t[0], w2t[1], w2t[2], w2t[3]);
      const s4 w2s = w2b;
#pragma unroll
      for (int i = 0; i < 4; ++i) W2mb[(4 * q + i) * LD2 + c] = (unsigned short)w2s[i];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) W2m[(4 * q + i) * LD2 + c] = w2t[i];  // W2[class c][unit 4q + s] at c*LD2 + 4q + s
    }
  };
  mirror();
  if (q == 0) B2m[c] = BF ? bfr(b2c) : b2c;

  // last step's (averaged) gradients, written to the DDP bucket at the end
  float lg1[MT][4], lg2[4], ldb2 = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    lg2[i] = 0.f;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) lg1[mt][i] = 0.f;
  }
  int ce = ce0, cj = cj0;  // current position (epoch, step in epoch): no divisions in the loop
  int sc = 0;              // LDS slot of the current batch
  constexpr bool stamps = ST;  // s_memtime is scalar: every wave times, thread 0 reports
  int64_t tmark = stamps ? (int64_t)__builtin_amdgcn_s_memtime() : 0;
  int64_t acc_t[7] = {0, 0, 0, 0, 0, 0, 0};
  int64_t acc_bar = 0;
  const int64_t t_begin = tmark, r_begin = stamps ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
  auto tick = [&](int ph) {
    if (stamps) {
      const int64_t t = (int64_t)__builtin_amdgcn_s_memtime();
      acc_t[ph] += t - tmark;
      tmark = t;
    }
  };
  for (int k = 0; k < n; ++k) {
    const int par = k & 1;
    const bool wrap = cj + 1 == S;
    const int ne = wrap ? ce + 1 : ce, nj = wrap ? 0 : cj + 1;
    const int sn = sc == 2 ? 0 : sc + 1;
    const int nb = min(B, ns - cj * B);
    const float* const st = stage(sc);

    // ---------------- fwd1: HT = W1aug . Xaug^T (this wave's 16 units x 32 rows), ReLU
    f4 h[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    if constexpr (BF) {  // one K = 32 MFMA per row tile (B: X row 16 t + c, inputs at tp_bpos)
      const unsigned short* const sb = reinterpret_cast<const unsigned short*>(st);
#pragma unroll
      for (int t = 0; t < 2; ++t)
        h[t] = mfma_k32(w1b, *reinterpret_cast<const bf8*>(sb + (16 * t + c) * LDX + 8 * q), h[t]);
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const f4 xb = *reinterpret_cast<const f4*>(st + (16 * t + c) * LDX + 16 * mt + 4 * q);
#pragma unroll
          for (int s = 0; s < (mt == MT - 1 ? KL : 4); ++s) h[t] = mfma4(w1r[mt][s], xb[s], h[t]);
        }
      }
    }
    float ht[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) ht[t][i] = fmaxf(h[t][i], 0.f);

    // ---------------- fwd2 partial: ZT_w = W2[:, slice] . HT (K steps permuted: unit 4q + s)
    f4 z[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    if constexpr (BF) {
      // B: bf16(H^T) in fwd1's result layout (K = the wave's 16 units)
      const s4 a2 = *reinterpret_cast<const s4*>(W2mb + c * LD2 + 4 * q);
#pragma unroll
      for (int t = 0; t < 2; ++t) z[t] = mfma_k16(a2, pack_bf4(ht[t][0], ht[t][1], ht[t][2], ht[t][3]), z[t]);
    } else {
      const f4 a2 = *reinterpret_cast<const f4*>(W2m + c * LD2 + 4 * q);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        z[0] = mfma4(a2[s], ht[0][s], z[0]);
        z[1] = mfma4(a2[s], ht[1][s], z[1]);
      }
    }
    {
      // tile-major planes: consecutive lanes read consecutive 16 B (no bank conflicts)
      f4* dst = reinterpret_cast<f4*>(xbuf + (par * NW + w) * 512 + l * 4);
      dst[0] = z[0];
      dst[64] = z[1];
    }
    // H^T of the slice for the backward's transposed reads (wave-private). Rows of the two tiles
    // interleave (batch row 16 t + c at position 2 c + t): one 8-B store per unit instead of two
    // 4-B stores, and the readers still fetch 8 consecutive positions with two 16-B loads
    // (BF: bf16 [16 units][kTpLB], the same positions = tp_rpos, one 4-B store per unit)
    if constexpr (BF) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned short*>(Th) + (4 * q + i) * kTpLB + 2 * c) =
            pack_bf16x2(ht[0][i], ht[1][i]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) *reinterpret_cast<f2*>(Th + (4 * q + i) * LDT + 2 * c) = f2{ht[0][i], ht[1][i]};
    }
    // ---- the loss is split by rows: wave w owns the 8-row slices sl = w, w + NW, .. (lane: row
    // lrow = l >> 3 of the slice, classes 2 lk, 2 lk + 1 with lk = l & 7), so the softmax is computed
    // once per element instead of once per wave; the dZ slices meet in LDS at a second barrier.
    // Everything the loss reads besides the partial logits is read before the first barrier: b2
    // (this wave's mirror) and the current batch's targets (staged in slot sc before the last barrier).
    const float* const ys = st + St::Y_OFF;
    const int lrow = l >> 3, lk = l & 7, cls0 = 2 * lk;  // (lr is the learning rate)
    constexpr int NSL = 4;  // 8-row slices of the 32-row tile pair
    const f2 b2v = *reinterpret_cast<const f2*>(B2m + cls0);
    int ylab[NSL];
    f2 ytg[NSL];
#pragma unroll
    for (int u = 0; u < NSL; ++u) {
      const int sl = w + u * NW;
      if (sl < NSL) {
        const int R = 8 * sl + lrow;
        if constexpr (LOSS == kLossCEIndex) ylab[u] = reinterpret_cast<const int*>(ys)[R];
        else ytg[u] = *reinterpret_cast<const f2*>(ys + R * 16 + cls0);
      }
    }
    // rows that take part (CE index: label not ignored), counted by every wave over all 32 rows
    float inv;
    bool none = false;
    if constexpr (LOSS == kLossCEIndex) {
      const int y32 = reinterpret_cast<const int*>(ys)[l & 31];
      const int cnt = __popcll(__ballot(l < 32 && l < nb && y32 != a.ignore_index));
      inv = cnt == B ? inv_full : 1.f / (float)(cnt > 0 ? cnt : 1);
      none = cnt == 0;
    } else {
      inv = nb == B ? inv_full : 1.f / (float)(LOSS == kLossMSE ? nb * Dout : nb);
    }
    tick(1);
    __syncthreads();
    if constexpr (ST) {  // the barrier alone (per wave, stamps[13 + w])
      const int64_t t = (int64_t)__builtin_amdgcn_s_memtime();
      acc_bar += t - tmark;
      tmark = t;
    }
#pragma unroll
    for (int u = 0; u < NSL; ++u) {
      const int sl = w + u * NW;  // uniform
      if (sl >= NSL) break;
      const int R = 8 * sl + lrow, tr = R >> 4, cr = R & 15;
      // logits: b2 + the NW partials in wave order (partials: lane (c', q') of tile tr holds
      // classes 4q'..4q'+3 of row c'); all reads in flight before the first add
      f2 pz[4];
#pragma unroll
      for (int v = 0; v < 4; ++v)
        if (v < NW)
          pz[v] = *reinterpret_cast<const f2*>(xbuf + (par * NW + v) * 512 + tr * 256 + ((lk >> 1) * 16 + cr) * 4 +
                                                2 * (lk & 1));
      f2 z = b2v;
#pragma unroll
      for (int v = 0; v < 4; ++v)
        if (v < NW) z += pz[v];
      if constexpr (BF) {  // autocast: the second Linear's output is bf16 (then CE in fp32)
        const uint32_t zz = pack_bf16x2(z[0], z[1]);
        z = f2{__uint_as_float(zz << 16), __uint_as_float(zz & 0xffff0000u)};
      }
      const bool rv = R < nb, ok0 = cls0 < Dout, ok1 = cls0 + 1 < Dout;
      float g0, g1, ls;
      if constexpr (LOSS == kLossMSE) {
        const f2 y = ytg[u];
        const float d0 = z[0] - y[0], d1 = z[1] - y[1];
        g0 = (rv && ok0) ? 2.f * d0 : 0.f;
        g1 = (rv && ok1) ? 2.f * d1 : 0.f;
        ls = ((rv && ok0) ? d0 * d0 : 0.f) + ((rv && ok1) ? d1 * d1 : 0.f);
      } else {
        float m = fmaxf(ok0 ? z[0] : -INFINITY, ok1 ? z[1] : -INFINITY);
        m = fmaxf(m, dpp_f<kDppXor1>(m));
        m = fmaxf(m, dpp_f<kDppXor2>(m));
        m = fmaxf(m, dpp_f<kDppHalfMirror>(m));
        const float e0 = ok0 ? __builtin_amdgcn_exp2f((z[0] - m) * 1.4426950408889634f) : 0.f;
        const float e1 = ok1 ? __builtin_amdgcn_exp2f((z[1] - m) * 1.4426950408889634f) : 0.f;
        const float se = group_sum<8>(e0 + e1);
        const float rse = __builtin_amdgcn_rcpf(se);  // softmax = e / se (v_rcp_f32); the log only feeds the loss
        const float lse = m + __builtin_amdgcn_logf(se) * 0.6931471805599453f;
        if constexpr (BF) {
          // torch.autocast(bfloat16) runs F.cross_entropy on bf16 logits as a bf16 log_softmax (fp32
          // inside, bf16 out), the nll / soft-target sum in fp32 on those bf16 values, and the backward
          // as a bf16 log_softmax_backward: dz = bf16(g - exp(ls) sum(g)) with g = bf16(dL/dls)
          // (measured: scripts/r6/ce_probe.py -- the autocast gradient equals the bf16-math one exactly)
          const float lg = __builtin_amdgcn_logf(se) * 0.6931471805599453f;
          const float l0 = ok0 ? bfr((z[0] - m) - lg) : 0.f, l1 = ok1 ? bfr((z[1] - m) - lg) : 0.f;
          const float p0 = ok0 ? __builtin_amdgcn_exp2f(l0 * 1.4426950408889634f) : 0.f;
          const float p1 = ok1 ? __builtin_amdgcn_exp2f(l1 * 1.4426950408889634f) : 0.f;
          float q0, q1, sg;
          if constexpr (LOSS == kLossCEIndex) {
            const int y = ylab[u];
            const bool use = rv && y != a.ignore_index;
            const float bi = bfr(inv);
            q0 = (use && cls0 == y) ? -bi : 0.f;
            q1 = (use && cls0 + 1 == y) ? -bi : 0.f;
            sg = use ? -bi : 0.f;
            g0 = (use && ok0) ? q0 - p0 * sg : 0.f;
            g1 = (use && ok1) ? q1 - p1 * sg : 0.f;
            ls = (use && cls0 == y) ? -l0 : ((use && cls0 + 1 == y) ? -l1 : 0.f);
          } else {
            const f2 y = ytg[u];
            q0 = (rv && ok0) ? bfr(-y[0] * inv) : 0.f;
            q1 = (rv && ok1) ? bfr(-y[1] * inv) : 0.f;
            sg = group_sum<8>(q0 + q1);
            g0 = (rv && ok0) ? q0 - p0 * sg : 0.f;
            g1 = (rv && ok1) ? q1 - p1 * sg : 0.f;
            ls = rv ? ((ok0 ? -y[0] * l0 : 0.f) + (ok1 ? -y[1] * l1 : 0.f)) : 0.f;
          }
        } else if constexpr (LOSS == kLossCEIndex) {
          const int y = ylab[u];
          const bool use = rv && y != a.ignore_index;
          g0 = (use && ok0) ? e0 * rse - (cls0 == y ? 1.f : 0.f) : 0.f;
          g1 = (use && ok1) ? e1 * rse - (cls0 + 1 == y ? 1.f : 0.f) : 0.f;
          ls = (use && cls0 == y) ? lse - z[0] : ((use && cls0 + 1 == y) ? lse - z[1] : 0.f);
        } else {  // soft targets: -(t . log_softmax(z)), grad = softmax * sum(t) - t
          const f2 y = ytg[u];  // classes >= Dout stage as 0
          const float sc = group_sum<8>(y[0] + y[1]) * rse;
          g0 = (rv && ok0) ? e0 * sc - y[0] : 0.f;
          g1 = (rv && ok1) ? e1 * sc - y[1] : 0.f;
          ls = rv ? ((ok0 ? -y[0] * (z[0] - lse) : 0.f) + (ok1 ? -y[1] * (z[1] - lse) : 0.f)) : 0.f;
        }
      }
      if constexpr (!BF || LOSS == kLossMSE) {  // (BF cross-entropy: 1/rows folded into g above)
        g0 *= inv;
        g1 *= inv;
      }
      // the row's loss (its 8 lanes' parts) into the loss ring: entry R of the step's 64 (32..63 stay 0)
      ls = group_sum<8>(ls);
      if (lk == 0) lring[(k & (kTpLossRing - 1)) * 64 + R] = (LOSS == kLossCEIndex && none) ? NAN : ls * inv;
      // dZ for every wave: row-major (dH's A operand) and transposed with interleaved tiles (row
      // 16 t + c at position 2 c + t; dW2's A operand and db2)
      if constexpr (BF) {  // bf16 dZ (autocast: the fp32 CE gradient cast back to the logits' dtype)
        const uint32_t gp = pack_bf16x2(g0, g1);
        *reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned short*>(dZr) + R * kTpLDZB + cls0) = gp;
        unsigned short* const zt = reinterpret_cast<unsigned short*>(dZt);
        zt[cls0 * kTpLB + tp_rpos(R)] = (unsigned short)gp;
        zt[(cls0 + 1) * kTpLB + tp_rpos(R)] = (unsigned short)(gp >> 16);
      } else {
        *reinterpret_cast<f2*>(dZr + R * kTpLDZ + cls0) = f2{g0, g1};
        dZt[cls0 * LDT + 2 * cr + tr] = g0;
        dZt[(cls0 + 1) * LDT + 2 * cr + tr] = g1;
      }
    }
    tick(2);
    __syncthreads();  // barrier 2: every slice of dZ is in LDS
    float g[2][4];
    s4 gA[2];  // BF: dH's A operand, dZ[row 16 t + c][class 4q + j] (8-B reads)
    if constexpr (BF) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
        gA[t] = *reinterpret_cast<const s4*>(reinterpret_cast<const unsigned short*>(dZr) + (16 * t + c) * kTpLDZB + 4 * q);
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const f4 gg = *reinterpret_cast<const f4*>(dZr + (16 * t + c) * kTpLDZ + 4 * q);
#pragma unroll
        for (int i = 0; i < 4; ++i) g[t][i] = gg[i];
      }
    }
    tick(3);

    // ---------------- dH = dZ . W2[:, slice]: dZ's result layout is the A operand
    // (row c, class 4q + s) and w2t the B operand (class 4q + s, unit c); the result
    // dH[row 16t + 4q + i][unit c] is dW1's B operand as it stands
    f4 gw2 = {0.f, 0.f, 0.f, 0.f};
    f4 gw1[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) gw1[mt] = f4{0.f, 0.f, 0.f, 0.f};
    float db2;
    if constexpr (BF) {
      // one K = 16 MFMA per row tile: A = dZ rows (gA), B = W2[class 4q + j][unit c] (w2b)
      const unsigned short* const sb = reinterpret_cast<const unsigned short*>(st);
      bf8 xa[MT];  // dW1's A: X^T[input 16 mt + c][rows at tp_rpos] (read now: hides under dH)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        xa[mt] = *reinterpret_cast<const bf8*>(sb + 2 * St::XT_OFF + (16 * mt + c) * LDXT + 8 * q);
      f4 dh[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) dh[t] = mfma_k16(gA[t], w2b, f4{0.f, 0.f, 0.f, 0.f});
      // H^T and dZ^T images (rows at tp_rpos): element j = row 16 (j & 1) + 4q + (j >> 1), i.e.
      // dh[j & 1][j >> 1] -- the ReLU mask, dW2's B and A
      const bf8 hT8 = *reinterpret_cast<const bf8*>(reinterpret_cast<const unsigned short*>(Th) + c * kTpLB + 8 * q);
      const bf8 dz8 = *reinterpret_cast<const bf8*>(reinterpret_cast<const unsigned short*>(dZt) + c * kTpLB + 8 * q);
      const s8 hraw = __builtin_bit_cast(s8, hT8);
      float dv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) dv[j] = hraw[j] > 0 ? dh[j & 1][j >> 1] : 0.f;  // bf16(H) > 0 (autocast's mask)
      const bf8 dH8 = pack_bf8(dv);  // autocast: dH in bf16
      const s8 zraw = __builtin_bit_cast(s8, dz8);
      float zf[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) zf[j] = __uint_as_float((uint32_t)(uint16_t)zraw[j] << 16);
      // db2[class c] = column sum of the bf16 dZ^T: this lane's 8 rows, then the 4 lane groups
      db2 = rows4_sum(((zf[0] + zf[1]) + (zf[2] + zf[3])) + ((zf[4] + zf[5]) + (zf[6] + zf[7])));
      // dW2 = dZ^T . H and dW1aug^T = Xaug^T . dH: one K = 32 MFMA per 16x16 result tile
      gw2 = mfma_k32(dz8, hT8, gw2);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) gw1[mt] = mfma_k32(xa[mt], dH8, gw1[mt]);
    } else {
      // X^T operands of dW1 (read now: their latency hides under the dH MFMAs)
      f4 xa[2][MT];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          xa[t][mt] = *reinterpret_cast<const f4*>(st + St::XT_OFF + (16 * mt + 4 * (c & 3) + (c >> 2)) * LDXT + 16 * t + 4 * q);
      f4 dh[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        dh[0] = mfma4(g[0][s], w2t[s], dh[0]);
        dh[1] = mfma4(g[1][s], w2t[s], dh[1]);
      }
      // transposed reads: H[row 16t + 4q + s][unit c] (ReLU mask, dW2's B) and
      // dZ[row 16t + 4q + s][class c] (dW2's A); interleaved tiles: positions 8q .. 8q+7 hold
      // rows 16t + 4q + s at 2s + t
      f4 hT[2], dzT[2];
      {
        const f4 h0 = *reinterpret_cast<const f4*>(Th + c * LDT + 8 * q);
        const f4 h1 = *reinterpret_cast<const f4*>(Th + c * LDT + 8 * q + 4);
        const f4 d0 = *reinterpret_cast<const f4*>(dZt + c * LDT + 8 * q);
        const f4 d1 = *reinterpret_cast<const f4*>(dZt + c * LDT + 8 * q + 4);
        hT[0] = f4{h0[0], h0[2], h1[0], h1[2]};
        hT[1] = f4{h0[1], h0[3], h1[1], h1[3]};
        dzT[0] = f4{d0[0], d0[2], d1[0], d1[2]};
        dzT[1] = f4{d0[1], d0[3], d1[1], d1[3]};
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) dh[t][i] = hT[t][i] > 0.f ? dh[t][i] : 0.f;
      // db2[class c] = column sum of dZ^T: this lane's 8 rows, then the 4 lane groups
      db2 = ((dzT[0][0] + dzT[0][1]) + (dzT[0][2] + dzT[0][3])) + ((dzT[1][0] + dzT[1][1]) + (dzT[1][2] + dzT[1][3]));
      db2 = rows4_sum(db2);

      // ---------------- dW2 = dZ^T . H (K = rows), dW1aug^T = Xaug^T . dH (K = rows)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          gw2 = mfma4(dzT[t][s], hT[t][s], gw2);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) gw1[mt] = mfma4(xa[t][mt][s], dh[t][s], gw1[mt]);
        }
      }
    }
    mfma_settle();  // uniform branches follow (hb, tick, the all-reduce's failed check)
    tick(4);

    // ---------------- all-reduce over ranks (xGMI LL), then SGD in registers
    float gv1[MT][4], gv2[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      gv2[i] = gw2[i];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) gv1[mt][i] = gw1[mt][i];
    }
    if constexpr (BF) {  // autocast: the weight / bias gradients of bf16 Linear ops are bf16
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        gv2[i] = bfr(gv2[i]);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) gv1[mt][i] = bfr(gv1[mt][i]);
      }
      db2 = bfr(db2);
    }
    if constexpr (AR) {
      if (!failed) {
        seq += 1u;
        constexpr int NV = 4 * MT + 5;
        float v[NV];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) v[mt * 4 + i] = gv1[mt][i];
          v[4 * MT + i] = gv2[i];
        }
        v[4 * MT + 4] = db2;  // b2[class c]: the same value in every wave (identical loss in every wave)
        // polls of G peers in flight (fp32: 3 where the registers allow it; bf16 packs two values
        // per word, so twice the peers fit: W = 8's seven peers in ceil(7 / G) rounds)
        constexpr int G = BF ? ((VX && LOSS == kLossCEIndex) ? kTpBfPollPeers : 4)
                             : ((LOSS == kLossCEIndex && VX) ? 3 : 2);
        failed = !tp_allreduce_lm<NV, G, BF>(a.ar, seq, v, w, l);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) gv1[mt][i] = v[mt * 4 + i];
          gv2[i] = v[4 * MT + i];
        }
        db2 = v[4 * MT + 4];
      }
    }
    tick(6);  // the all-reduce alone (0 at world 1; index 6 was the list producer before the helper wave)
    // padded inputs / classes have zero gradients and zero weights: no masks needed
    const bool first = opt_step == 0;
    if (plain_sgd) {  // (uniform) the reference's SGD(lr): one FMA per value, no momentum / decay chain
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) w1r[mt][i] = fmaf(-lr, gv1[mt][i], w1r[mt][i]);
        w2t[i] = fmaf(-lr, gv2[i], w2t[i]);
      }
      if (hb) b2c = fmaf(-lr, db2, b2c);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) sgd1(w1r[mt][i], m1r[mt][i], gv1[mt][i], first, lr, mu, damp, wd, nesterov, use_mom);
        sgd1(w2t[i], m2t[i], gv2[i], first, lr, mu, damp, wd, nesterov, use_mom);
      }
      if (hb) sgd1(b2c, mb2c, db2, first, lr, mu, damp, wd, nesterov, use_mom);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) lg1[mt][i] = gv1[mt][i];
      if constexpr (!BF) W2m[(4 * q + i) * LD2 + c] = w2t[i];
      lg2[i] = gv2[i];
    }
    if constexpr (BF) mirror();  // bf16 operand copies of the updated weights
    if (hb && q == 0) B2m[c] = BF ? bfr(b2c) : b2c;  // (no bias: b2c and its gradient stay 0)
    ldb2 = db2;
    ++opt_step;
    ce = ne;
    cj = nj;
    sc = sn;
    tick(5);
  }
  if (n > 0) __syncthreads();  // the helper's final flush reads every step's loss share

  // ---- write back: parameters, momentum, the last step's averaged gradients (DDP bucket)
  float* const Pw = a.P;
  float* const Gw = a.G;
  const bool have = n > 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int in = BF ? 16 * mt + 4 * q + i : 16 * mt + 4 * i + q;
      const int off = in < Din ? d.oW1 + unit * Din + in : (hb && in == Din ? d.ob1 + unit : -1);
      if (off >= 0) {
        Pw[off] = w1r[mt][i];
        if (use_mom) a.mom[off] = m1r[mt][i];
        if (have) Gw[off] = lg1[mt][i];
      }
    }
    const int cls = 4 * q + i;
    if (cls < Dout) {
      const int off = d.oW2 + cls * H + unit;
      Pw[off] = w2t[i];
      if (use_mom) a.mom[off] = m2t[i];
      if (have) Gw[off] = lg2[i];
    }
  }
  if (hb && q == 0 && w == 0 && c < Dout) {
    Pw[d.ob2 + c] = b2c;
    if (use_mom) a.mom[d.ob2 + c] = mb2c;
    if (have) Gw[d.ob2 + c] = ldb2;
  }
  if (stamps && l == 0 && pa.stamps_n >= 13 + NW) {  // each wave's logit-sum phase and barrier wait
    pa.stamps[9 + w] += acc_t[2];
    pa.stamps[13 + w] += acc_bar;
  }
  if (tid == 0) {
    pa.cursor[0] = ce;
    pa.cursor[1] = cj;
    if (stamps) {  // [0] - (helper wave) [1] fwd [2] barrier+sum [3] loss [4] bwd MFMA [5] SGD [6] all-reduce
      for (int k = 0; k < 7; ++k) pa.stamps[k] += acc_t[k];
      pa.stamps[7] += (int64_t)__builtin_amdgcn_s_memtime() - t_begin;
      pa.stamps[8] += (int64_t)__builtin_amdgcn_s_memrealtime() - r_begin;
      // prologue marks relative to kernel entry: [17] lists/init [18] barrier [19] staged, [20] state
      // loaded [21] list e0 [22] list e0+1 + keys
      if (pa.stamps_n >= 23)
        for (int k = 0; k < 3; ++k) {
          pa.stamps[17 + k] += r_pro[3 + k] - r_entry;
          pa.stamps[20 + k] += r_pro[k] - r_entry;
        }
    }
    if (a.opt_step) *a.opt_step = opt_step;
    if (AR) *a.ar.seq = seq;
  }
}

int tp_mt(const FusedMlpArgs& a) { return a.Din + (a.has_bias ? 1 : 0) <= 16 ? 1 : 2; }

bool tp_vec_x(const FusedMlpArgs& a) {
  const int ldx = a.ldx > 0 ? a.ldx : a.Din;
  return a.Din % 4 == 0 && ldx % 4 == 0 && reinterpret_cast<uintptr_t>(a.X) % 16 == 0;
}

size_t tp_lds_bytes(const FusedMlpArgs& a, const PersistArgs& p, bool bf) {
  const int NW = a.H / 16;
  const size_t fl = (size_t)3 * al4(p.num_samples) + (size_t)3 * tp_stage_floats(tp_mt(a), bf) +
                    (size_t)2 * NW * 64 * 8 + (size_t)NW * tp_wave_floats() + 48 + 3 + (size_t)kTpLossRing * 64 +
                    (size_t)32 * kTpLDZ + (size_t)16 * kTpLDT;
  return fl * sizeof(float);
}

}  // namespace

// the bf16-operand instantiations (mlp_tp_bf16.hip); mt: dW1's 16-input result tiles (1 or 2)
const void* mlp_tp_bf16_kernel(int loss, bool ar, bool vx, int mt, bool st);

}  // namespace ptdt
