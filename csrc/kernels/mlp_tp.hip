// Persistent DDP step engine for Linear(Din,H)-ReLU-Linear(H,Dout) + loss + SGD,
// tensor-parallel across the waves of ONE workgroup, every product on MFMA.
//
// The toy MLP of BASELINE.json's north star (Linear(20,64)-ReLU-Linear(64,10),
// CE, SGD; per-device batch 32 as in ddp_gpus.py:34-39) is ~143K MACs per step:
// a latency problem, not a throughput one. Round 1's workgroup engine ran the
// step as LDS-staged phases separated by workgroup barriers (~15K cycles per
// step, MFMA ~2K of it). Here each of NW = H/16 waves owns 16 hidden units --
// its slice of W1, b1 and the matching columns of W2, master copies + momentum
// in its own LDS region / registers -- and runs its whole slice of the step
// with v_mfma_f32_16x16x4_f32 (exact fp32, 32 cycles per SIMD):
//
//   fwd1  HT[j][r]   = W1[j][:] . X[r][:]           (K = Din,  A: LDS W1, B: X rows)
//   fwd2  ZT_w[c][r] = W2[c][slice] . HT[slice][r]   (K = the wave's 16 units; the
//         MFMA D layout of HT (m on lane>>4, reg) IS the B operand with the K steps
//         permuted to k = 4*(lane>>4) + s: no data movement)
//   ----  ONE workgroup barrier per step: the NW partial logits meet in LDS and
//         every wave sums them in wave order (identical bits in every wave)
//   loss  softmax / CE / MSE on the D layout: classes across the 4 lane groups
//         (permlane16/32 swaps), rows across the 16 lanes; every wave computes it
//   dHT   = W2[:, slice]^T . dZT                     (K = classes, same trick)
//   dW2, dW1^T need K = rows: HT, dZT, dHT go through a wave-private LDS
//         transpose (no barrier: one wave's LDS ops complete in order)
//   SGD   on the wave's slice (W1/W2 in LDS, biases in registers)
//
// so a step is ~50 MFMAs per wave on 4 SIMDs in parallel plus one barrier,
// instead of phase-by-phase work over shared LDS. Batches are gathered from the
// device-resident dataset one step ahead straight into MFMA operand registers.
// Sampler lists live in LDS (three epoch slots); the entries of each future
// position are produced S+1 steps ahead of their use, C = min(8, S) positions at a
// time by all threads, so epoch transitions cost nothing. With an all-reduce (world > 1) every lane
// exchanges its gradient registers over xGMI with the LL protocol of
// comm/xgmi.h (push to every peer, poll, sum in rank order: bit-identical
// replicas), then applies SGD.
#include "common.h"
#include "kernels.h"
#include "sampler.h"

namespace ptdt {
namespace {

constexpr int kTpThreadsMax = 256;
using f4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

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
  int B, Din, H, Dout, NW, KS1, ld1, ld2, ldT, estride;
  int oW1, ob1, oW2, ob2, np;
};

__device__ __forceinline__ TpDims tp_dims(const FusedMlpArgs& a, const PersistArgs& pa) {
  TpDims d;
  d.B = a.B; d.Din = a.Din; d.H = a.H; d.Dout = a.Dout;
  d.NW = a.H / 16;
  d.KS1 = (a.Din + 3) / 4;
  d.ld1 = 4 * d.KS1 + 1;  // W1 slice row stride (units x padded inputs)
  d.ld2 = 17;             // W2 slice row stride (classes x 16 units)
  d.ldT = 33;             // transpose tiles: 16 x 32 rows
  d.estride = al4(pa.num_samples);
  const int hb = a.has_bias != 0;
  d.oW1 = 0;
  d.ob1 = a.H * a.Din;
  d.oW2 = d.ob1 + (hb ? a.H : 0);
  d.ob2 = d.oW2 + a.Dout * a.H;
  d.np = d.ob2 + (hb ? a.Dout : 0);
  return d;
}

// floats of LDS per wave: W1, M1 (16 x ld1), W2, M2 (16 x ld2), 3 transpose tiles (16 x ldT)
__host__ __device__ __forceinline__ int tp_wave_floats(int KS1) {
  return 2 * 16 * (4 * KS1 + 1) + 2 * 16 * 17 + 3 * 16 * 33;
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

// Gradient all-reduce of NV register values over xGMI (LL words, comm/xgmi.h):
// push[k] lanes send value k (flat index idx[k]) to every peer, then every lane
// with need[k] polls the W contributions and sums them in rank order (its own
// from the register). Returns false after a poll timeout (and sets *err).
template <int NV>
__device__ __forceinline__ bool tp_allreduce(const XgmiArgs& x, uint32_t seq, float (&v)[NV], const int (&idx)[NV],
                                             const bool (&push)[NV], const bool (&need)[NV]) {
  const int parity = (int)(seq & 1u);
  const uint64_t hi = (uint64_t)seq << 32;
  const bool drop = x.drop_push != 0u && seq >= x.drop_push;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    if (!push[k] || drop) continue;
    const uint64_t w = hi | (uint64_t)__float_as_uint(v[k]);
    for (int p = 0; p < x.world; ++p)
      if (p != x.rank)
        __hip_atomic_store(xgmi_slot(x.peers[p], parity, x.rank, x.world, x.max_elems, idx[k]), w, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  }
  bool ok = true;
  float acc[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) acc[k] = 0.f;
  for (int p = 0; p < x.world; ++p) {
    if (p == x.rank) {
#pragma unroll
      for (int k = 0; k < NV; ++k) acc[k] += v[k];
      continue;
    }
    uint64_t w[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k)  // all polls of this peer in flight together
      w[k] = need[k] ? __hip_atomic_load(xgmi_slot(x.local, parity, p, x.world, x.max_elems, idx[k]), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM)
                     : hi;
    for (uint32_t polls = 0;; ++polls) {
      bool all = true;
#pragma unroll
      for (int k = 0; k < NV; ++k) all &= (uint32_t)(w[k] >> 32) == seq;
      if (all) break;
      if (polls >= x.max_polls) {
        __hip_atomic_store(x.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
#pragma unroll
      for (int k = 0; k < NV; ++k)
        if ((uint32_t)(w[k] >> 32) != seq)
          w[k] = __hip_atomic_load(xgmi_slot(x.local, parity, p, x.world, x.max_elems, idx[k]), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (!ok) break;
#pragma unroll
    for (int k = 0; k < NV; ++k) acc[k] += need[k] ? __uint_as_float((uint32_t)w[k]) : 0.f;
  }
  const float inv = 1.f / (float)x.world;
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = acc[k] * inv;
  return ok;
}

// One batch in MFMA operand registers.
template <int MT>
struct TpBatch {
  float xb[2][8];   // fwd1 B operand (first KS used): X[row 16t + c][in 4s + q] (0 for in >= Din)
  float xa[MT][8];  // dW1^T A operand: X[row 4s + q][in 16mt + c] (0 for in >= Din)
  float yf[2][4];   // soft / MSE targets (row 16t + c, class 4q + i)
  int yi[2];        // class labels of rows 16t + c
  int nb;           // valid rows of this batch
};

// KS: fwd1 K steps (4 inputs each; Din <= 4 KS, padded with zeros), MT = input tiles of dW1^T
template <int KS, int LOSS, bool AR>
__global__ void __launch_bounds__(kTpThreadsMax) mlp_tp_kernel(FusedMlpArgs a, PersistArgs pa) {
  // No implicit FMA contraction: the compiler may contract differently in a peeled
  // first iteration than in the loop body, which made a run split into several
  // launches differ in the last bit from one long launch. Fused ops are explicit
  // (fmaf in sgd1, MFMA).
#pragma clang fp contract(off)
  constexpr int MT = KS > 4 ? 2 : 1;
  constexpr int LD1 = 4 * KS + 1;  // W1 slice row stride (units x padded inputs)
  constexpr int LD2 = 17, LDT = 33;
  extern __shared__ float lds[];
  const TpDims d = tp_dims(a, pa);
  const int tid = (int)threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l = tid & 63, c = l & 15, q = l >> 4;
  const int B = d.B, Din = d.Din, H = d.H, Dout = d.Dout, NW = d.NW;
  const bool hb = a.has_bias != 0;
  const bool use_mom = a.mom != nullptr && a.momentum != 0.f;
  const float lr = a.lr, mu = a.momentum, damp = a.dampening, wd = a.weight_decay;
  const int nesterov = a.nesterov;

  // ---- LDS carve-up
  // [3][estride] epoch lists: a producer one epoch ahead never overwrites a list a
  // lagging wave may still read (position P's and P+1's epochs)
  int* const elist = reinterpret_cast<int*>(lds);
  float* const xbuf = lds + 3 * d.estride;                           // [2][NW][64][8] partial logits
  float* const wbase = xbuf + 2 * NW * 64 * 8 + tp_wave_floats(KS) * w;
  float* const W1m = wbase;                      // [16][ld1] this wave's W1 rows (units 16w..16w+15)
  float* const M1m = W1m + 16 * LD1;
  float* const W2m = M1m + 16 * LD1;           // [16 classes][ld2] columns 16w..16w+15 of W2
  float* const M2m = W2m + 16 * LD2;
  float* const Tdz = M2m + 16 * LD2;           // [16][ldT] transposes: dZT, HT, dHT (class/unit x row)
  float* const Th = Tdz + 16 * LDT;
  float* const Tdh = Th + 16 * LDT;
  auto list = [&](int e) { return elist + (e % 3) * d.estride; };

  // ---- sampler lists: epoch e0 whole, epoch e0+1 up to batch j0 (entries of later
  // positions are produced S+1 steps ahead inside the loop)
  const int ns = pa.num_samples;
  const int S = (ns + B - 1) / B;
  const int e0 = pa.cursor[0], j0 = pa.cursor[1];
  const int64_t pos0 = (int64_t)e0 * S + j0;
  const int n = pa.n_steps;
  const ListCache lc{pa.lcache, pa.ltag, d.estride};
  rank_epoch_indices_or(given_list(pa, e0), list(e0), (uint32_t)pa.N, pa.W, pa.rank, ns, pa.seed, e0, pa.shuffle, tid,
                        (int)blockDim.x, lc);
  {
    const int upto = min((j0 + 1) * B, ns);
    const int32_t* g1 = given_list(pa, e0 + 1);
    FeistelPerm fp;
    fp.init(pa.seed, e0 + 1, (uint32_t)pa.N);
    const uint32_t step_w = (uint32_t)pa.W;
    for (int i = tid; i < ns; i += (int)blockDim.x) {
      int v = 0;  // zero-filled beyond: stale prefetches past the launch read valid rows
      if (i < upto) {
        const uint32_t pos = (uint32_t)(((uint64_t)pa.rank + (uint64_t)step_w * (uint64_t)i) % (uint32_t)pa.N);
        v = g1 ? g1[i] : (int)(pa.shuffle ? fp(pos) : pos);
      }
      list(e0 + 1)[i] = v;
    }
  }
  __syncthreads();
  if (tid == 0 && pa.idx == nullptr) list_cache_publish(lc, e0);

  // Chunked producer: every C = min(8, S) steps ALL threads produce the entries of the
  // C positions S+1 .. S+C ahead (one entry per thread for B <= 32), so the cycle-
  // walking Feistel of the device sampler costs one evaluation per thread per C steps
  // on every wave alike. Produced lists are not cached (the cache only holds lists
  // computed whole by a prologue); three LDS slots keep any produced epoch clear of
  // the epochs still read (positions P and P+1).
  const int C = min(8, S);
  auto produce = [&](int te, int tj) {  // positions (te, tj) .. + C - 1
    for (int idx = tid; idx < C * B; idx += (int)blockDim.x) {
      const int o = idx / B, r = idx - o * B;
      int J = tj + o, E = te;
      if (J >= S) {
        J -= S;
        ++E;
      }
      const int i = J * B + r;
      if (i >= ns) continue;
      int v;
      if (pa.idx != nullptr) {
        v = given_list(pa, E)[i];
      } else {
        const uint32_t pos = (uint32_t)(((uint64_t)pa.rank + (uint64_t)pa.W * (uint64_t)i) % (uint32_t)pa.N);
        if (pa.shuffle) {
          FeistelPerm fp;
          fp.init(pa.seed, E, (uint32_t)pa.N);
          v = (int)fp(pos);
        } else {
          v = (int)pos;
        }
      }
      list(E)[i] = v;
    }
  };

  // ---- resident state
  const auto P = gptr(a.P);
  for (int e = l; e < 16 * LD1; e += 64) {
    const int j = e / LD1, in = e - j * LD1;
    const bool real = in < Din;
    W1m[e] = real ? P[d.oW1 + (16 * w + j) * Din + in] : 0.f;
    M1m[e] = (real && use_mom) ? a.mom[d.oW1 + (16 * w + j) * Din + in] : 0.f;
  }
  for (int e = l; e < 16 * LD2; e += 64) {
    const int cls = e / LD2, j = e - cls * LD2;
    const bool real = cls < Dout && j < 16;
    W2m[e] = real ? P[d.oW2 + cls * H + 16 * w + j] : 0.f;
    M2m[e] = (real && use_mom) ? a.mom[d.oW2 + cls * H + 16 * w + j] : 0.f;
  }
  float b1r[4], mb1r[4], b2r[4], mb2r[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int u = 16 * w + 4 * q + i, cls = 4 * q + i;
    b1r[i] = hb ? P[d.ob1 + u] : 0.f;
    mb1r[i] = (hb && use_mom) ? a.mom[d.ob1 + u] : 0.f;
    b2r[i] = (hb && cls < Dout) ? P[d.ob2 + cls] : 0.f;
    mb2r[i] = (hb && use_mom && cls < Dout) ? a.mom[d.ob2 + cls] : 0.f;
  }
  int opt_step = a.opt_step ? *a.opt_step : 0;
  uint32_t seq = AR ? *a.ar.seq : 0u;
  bool failed = AR && *a.ar.err != 0;

  // ---- batch fetch (next position's rows, straight into operand registers)
  const auto X = gptr(a.X);
  const int ldx = a.ldx > 0 ? a.ldx : Din;
  auto fetch = [&](TpBatch<MT>& f, int E, int J) {
    const int nb = min(B, ns - J * B);
    f.nb = nb;
    const int* li = list(E) + J * B;
    // unconditional loads (clamped indices) + selects: no per-element branches
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int sel = li[min(16 * t + c, nb - 1)];
      const auto xr = X + (int64_t)sel * ldx;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int in = 4 * s + q;
        const float v = xr[min(in, Din - 1)];
        f.xb[t][s] = in < Din ? v : 0.f;
      }
      if constexpr (LOSS == kLossCEIndex) {
        f.yi[t] = (int)gptr(a.Yi)[sel];
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int cls = 4 * q + i;
          const float v = gptr(a.Yf)[(int64_t)sel * Dout + min(cls, Dout - 1)];
          f.yf[t][i] = cls < Dout ? v : 0.f;
        }
      }
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int sel = li[min(4 * s + q, nb - 1)];
      const auto xr = X + (int64_t)sel * ldx;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int in = 16 * mt + c;
        const float v = xr[min(in, Din - 1)];
        f.xa[mt][s] = in < Din ? v : 0.f;
      }
    }
  };

  float* const losses = pa.losses;
  // last step's (averaged) gradients, written to the DDP bucket at the end
  float lg1[MT][4], lg2[4], ldb1[4], ldb2[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    lg2[i] = ldb1[i] = ldb2[i] = 0.f;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) lg1[mt][i] = 0.f;
  }

  TpBatch<MT> cur, nxt;
  fetch(cur, e0, j0);
  int ce = e0, cj = j0;  // current position (epoch, step in epoch): no divisions in the loop
  const bool stamps = pa.stamps != nullptr && tid == 0;
  int64_t tmark = stamps ? (int64_t)__builtin_amdgcn_s_memtime() : 0;
  int64_t acc_t[6] = {0, 0, 0, 0, 0, 0};
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
    fetch(nxt, ne, nj);  // stale-but-valid past the launch
    if (k % C == 0) produce(wrap ? ce + 2 : ce + 1, wrap ? 0 : cj + 1);
    tick(0);
    const int nb = cur.nb;

    // ---------------- fwd1: HT = W1 . X^T (this wave's 16 units x 32 rows)
    f4 h[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const float aw = W1m[c * LD1 + 4 * s + q];
      h[0] = mfma4(aw, cur.xb[0][s], h[0]);
      h[1] = mfma4(aw, cur.xb[1][s], h[1]);
    }
    float ht[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) ht[t][i] = fmaxf(h[t][i] + b1r[i], 0.f);

    // ---------------- fwd2 partial: ZT_w = W2[:, slice] . HT (K steps permuted: unit 4q + s)
    f4 z[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float a2 = W2m[c * LD2 + 4 * q + s];
      z[0] = mfma4(a2, ht[0][s], z[0]);
      z[1] = mfma4(a2, ht[1][s], z[1]);
    }
    {
      float4* dst = reinterpret_cast<float4*>(xbuf + ((par * NW + w) * 64 + l) * 8);
      dst[0] = make_float4(z[0][0], z[0][1], z[0][2], z[0][3]);
      dst[1] = make_float4(z[1][0], z[1][1], z[1][2], z[1][3]);
    }
    // the transposes of HT can go out while the other waves catch up
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) Th[(4 * q + i) * LDT + 16 * t + c] = ht[t][i];
    tick(1);
    __syncthreads();
    float zf[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) zf[t][i] = 0.f;
    for (int v = 0; v < NW; ++v) {  // wave order: identical sums in every wave
      const float4* src = reinterpret_cast<const float4*>(xbuf + ((par * NW + v) * 64 + l) * 8);
      const float4 p0 = src[0], p1 = src[1];
      zf[0][0] += p0.x; zf[0][1] += p0.y; zf[0][2] += p0.z; zf[0][3] += p0.w;
      zf[1][0] += p1.x; zf[1][1] += p1.y; zf[1][2] += p1.z; zf[1][3] += p1.w;
    }

    tick(2);
    // ---------------- loss and dL/dZ (classes 4q + i across lane groups, rows 16t + c)
    float g[2][4];
    float lsum = 0.f, cnt = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const bool rv = 16 * t + c < nb;
#pragma unroll
      for (int i = 0; i < 4; ++i) zf[t][i] += b2r[i];
      if constexpr (LOSS == kLossMSE) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bool ok = rv && 4 * q + i < Dout;
          const float df = zf[t][i] - cur.yf[t][i];
          lsum += ok ? df * df : 0.f;
          g[t][i] = ok ? 2.f * df : 0.f;
        }
      } else {
        float m = -INFINITY;
#pragma unroll
        for (int i = 0; i < 4; ++i) m = (4 * q + i < Dout) ? fmaxf(m, zf[t][i]) : m;
        m = rows4_max(m);
        float se = 0.f;
        float e[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          e[i] = (4 * q + i < Dout) ? __expf(zf[t][i] - m) : 0.f;
          se += e[i];
        }
        se = rows4_sum(se);
        const float lse = m + __builtin_amdgcn_logf(se) * 0.6931471805599453f;
        if constexpr (LOSS == kLossCEIndex) {
          const int y = cur.yi[t];
          const bool use = rv && y != a.ignore_index;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int cls = 4 * q + i;
            const float p = __expf(zf[t][i] - lse);
            g[t][i] = (use && cls < Dout) ? p - (cls == y ? 1.f : 0.f) : 0.f;
            lsum += (use && cls == y) ? lse - zf[t][i] : 0.f;
          }
          cnt += (use && q == 0) ? 1.f : 0.f;
        } else {  // soft targets: -(t . log_softmax(z)), grad = softmax * sum(t) - t
          float ts = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) ts += (4 * q + i < Dout) ? cur.yf[t][i] : 0.f;
          ts = rows4_sum(ts);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const bool ok = rv && 4 * q + i < Dout;
            const float ls = zf[t][i] - lse;
            lsum += ok ? -cur.yf[t][i] * ls : 0.f;
            g[t][i] = ok ? __expf(ls) * ts - cur.yf[t][i] : 0.f;
          }
        }
      }
    }
    float inv;
    if constexpr (LOSS == kLossCEIndex) {
      cnt = wave_sum(cnt);
      inv = 1.f / (cnt > 0.f ? cnt : 1.f);
    } else if constexpr (LOSS == kLossMSE) {
      inv = 1.f / (float)(nb * Dout);
    } else {
      inv = 1.f / (float)nb;
    }
    lsum = wave_sum(lsum);
    if (w == 0 && l == 0)
      losses[k] = (LOSS == kLossCEIndex && !(cnt > 0.f)) ? NAN : lsum * inv;
    float db2[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      g[0][i] *= inv;
      g[1][i] *= inv;
      db2[i] = group_sum<16>(g[0][i]) + group_sum<16>(g[1][i]);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) Tdz[(4 * q + i) * LDT + 16 * t + c] = g[t][i];

    tick(3);
    // ---------------- dHT = W2[:, slice]^T . dZT (K steps permuted: class 4q + s), ReLU mask
    f4 dh[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float a3 = W2m[(4 * q + s) * LD2 + c];
      dh[0] = mfma4(a3, g[0][s], dh[0]);
      dh[1] = mfma4(a3, g[1][s], dh[1]);
    }
    float db1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      dh[0][i] = ht[0][i] > 0.f ? dh[0][i] : 0.f;
      dh[1][i] = ht[1][i] > 0.f ? dh[1][i] : 0.f;
      db1[i] = group_sum<16>(dh[0][i]) + group_sum<16>(dh[1][i]);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) Tdh[(4 * q + i) * LDT + 16 * t + c] = dh[t][i];

    // ---------------- dW2 = dZT . H (K = rows), dW1^T = X^T . dH (K = rows)
    f4 gw2 = {0.f, 0.f, 0.f, 0.f};
    f4 gw1[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) gw1[mt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int r = 4 * s + q;
      const float adz = Tdz[c * LDT + r];
      const float bh = Th[c * LDT + r];
      const float bdh = Tdh[c * LDT + r];
      gw2 = mfma4(adz, bh, gw2);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) gw1[mt] = mfma4(cur.xa[mt][s], bdh, gw1[mt]);
    }

    tick(4);
    // ---------------- all-reduce over ranks (xGMI LL), then SGD on the slice
    float gv1[MT][4], gv2[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      gv2[i] = gw2[i];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) gv1[mt][i] = gw1[mt][i];
    }
    if constexpr (AR) {
      if (!failed) {
        seq += 1u;
        constexpr int NV = 4 * MT + 12;
        float v[NV];
        int idx[NV];
        bool push[NV], need[NV];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const int in = 16 * mt + 4 * q + i;
            const bool ok = in < Din;
            v[mt * 4 + i] = gv1[mt][i];
            idx[mt * 4 + i] = ok ? d.oW1 + (16 * w + c) * Din + in : 0;
            push[mt * 4 + i] = need[mt * 4 + i] = ok;
          }
          const int cls = 4 * q + i;
          v[4 * MT + i] = gv2[i];
          idx[4 * MT + i] = cls < Dout ? d.oW2 + cls * H + 16 * w + c : 0;
          push[4 * MT + i] = need[4 * MT + i] = cls < Dout;
          v[4 * MT + 4 + i] = db1[i];
          idx[4 * MT + 4 + i] = hb ? d.ob1 + 16 * w + 4 * q + i : 0;
          push[4 * MT + 4 + i] = hb && c == 0;
          need[4 * MT + 4 + i] = hb;
          v[4 * MT + 8 + i] = db2[i];
          idx[4 * MT + 8 + i] = (hb && cls < Dout) ? d.ob2 + cls : 0;
          push[4 * MT + 8 + i] = hb && cls < Dout && c == 0 && w == 0;
          need[4 * MT + 8 + i] = hb && cls < Dout;
        }
        failed = !tp_allreduce<NV>(a.ar, seq, v, idx, push, need);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) gv1[mt][i] = v[mt * 4 + i];
          gv2[i] = v[4 * MT + i];
          db1[i] = v[4 * MT + 4 + i];
          db2[i] = v[4 * MT + 8 + i];
        }
      }
    }
    const bool first = opt_step == 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int in = 16 * mt + 4 * q + i;
        if (in < Din) {
          const int e = c * LD1 + in;
          float wv = W1m[e], mv = M1m[e];
          sgd1(wv, mv, gv1[mt][i], first, lr, mu, damp, wd, nesterov, use_mom);
          W1m[e] = wv;
          M1m[e] = mv;
        }
        lg1[mt][i] = gv1[mt][i];
      }
      const int cls = 4 * q + i;
      if (cls < Dout) {
        const int e = cls * LD2 + c;
        float wv = W2m[e], mv = M2m[e];
        sgd1(wv, mv, gv2[i], first, lr, mu, damp, wd, nesterov, use_mom);
        W2m[e] = wv;
        M2m[e] = mv;
      }
      if (hb) {
        sgd1(b1r[i], mb1r[i], db1[i], first, lr, mu, damp, wd, nesterov, use_mom);
        if (cls < Dout) sgd1(b2r[i], mb2r[i], db2[i], first, lr, mu, damp, wd, nesterov, use_mom);
      }
      lg2[i] = gv2[i];
      ldb1[i] = db1[i];
      ldb2[i] = db2[i];
    }
    ++opt_step;
    cur = nxt;
    ce = ne;
    cj = nj;
    tick(5);
  }

  // ---- write back: parameters, momentum, the last step's averaged gradients (DDP bucket)
  __syncthreads();
  float* const Pw = a.P;
  float* const Gw = a.G;
  const bool have = n > 0;
  for (int e = l; e < 16 * Din; e += 64) {
    const int j = e / Din, in = e - j * Din;
    Pw[d.oW1 + (16 * w + j) * Din + in] = W1m[j * LD1 + in];
    if (use_mom) a.mom[d.oW1 + (16 * w + j) * Din + in] = M1m[j * LD1 + in];
  }
  for (int e = l; e < Dout * 16; e += 64) {
    const int cls = e / 16, j = e - cls * 16;
    Pw[d.oW2 + cls * H + 16 * w + j] = W2m[cls * LD2 + j];
    if (use_mom) a.mom[d.oW2 + cls * H + 16 * w + j] = M2m[cls * LD2 + j];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int cls = 4 * q + i;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int in = 16 * mt + 4 * q + i;
      if (have && in < Din) Gw[d.oW1 + (16 * w + c) * Din + in] = lg1[mt][i];
    }
    if (have && cls < Dout) Gw[d.oW2 + cls * H + 16 * w + c] = lg2[i];
    if (hb && c == 0) {
      Pw[d.ob1 + 16 * w + 4 * q + i] = b1r[i];
      if (use_mom) a.mom[d.ob1 + 16 * w + 4 * q + i] = mb1r[i];
      if (have) Gw[d.ob1 + 16 * w + 4 * q + i] = ldb1[i];
      if (w == 0 && cls < Dout) {
        Pw[d.ob2 + cls] = b2r[i];
        if (use_mom) a.mom[d.ob2 + cls] = mb2r[i];
        if (have) Gw[d.ob2 + cls] = ldb2[i];
      }
    }
  }
  if (tid == 0) {
    pa.cursor[0] = ce;
    pa.cursor[1] = cj;
    if (stamps) {  // [0] fetch+produce [1] fwd [2] barrier+sum [3] loss [4] bwd MFMA [5] all-reduce+SGD
      for (int k = 0; k < 6; ++k) pa.stamps[k] += acc_t[k];
      pa.stamps[7] += (int64_t)__builtin_amdgcn_s_memtime() - t_begin;
      pa.stamps[8] += (int64_t)__builtin_amdgcn_s_memrealtime() - r_begin;
    }
    if (a.opt_step) *a.opt_step = opt_step;
    if (AR) *a.ar.seq = seq;
  }
}

int tp_ks(int Din) { return Din <= 8 ? 2 : Din <= 16 ? 4 : Din <= 20 ? 5 : 8; }

template <int LOSS, bool AR>
const void* pick_ks(int ks) {
  switch (ks) {
    case 2: return (const void*)mlp_tp_kernel<2, LOSS, AR>;
    case 4: return (const void*)mlp_tp_kernel<4, LOSS, AR>;
    case 5: return (const void*)mlp_tp_kernel<5, LOSS, AR>;
    default: return (const void*)mlp_tp_kernel<8, LOSS, AR>;
  }
}

template <bool AR>
const void* pick_loss_tp(int loss, int ks) {
  switch (loss) {
    case kLossCEIndex: return pick_ks<kLossCEIndex, AR>(ks);
    case kLossMSE: return pick_ks<kLossMSE, AR>(ks);
    default: return pick_ks<kLossCESoft, AR>(ks);
  }
}

size_t tp_lds_bytes(const FusedMlpArgs& a, const PersistArgs& p) {
  const int NW = a.H / 16;
  const size_t fl = (size_t)3 * al4(p.num_samples) + (size_t)2 * NW * 64 * 8 + (size_t)NW * tp_wave_floats(tp_ks(a.Din));
  return fl * sizeof(float);
}

}  // namespace

bool mlp_tp_supported(const FusedMlpArgs& a, const PersistArgs& p) {
  if (a.H < 16 || a.H > 64 || a.H % 16 != 0) return false;
  if (a.B < 1 || a.B > 32 || a.Din < 1 || a.Din > 32 || a.Dout < 1 || a.Dout > 16) return false;
  if (a.ar.world > kXgmiMaxRanks) return false;
  if (p.N <= 0 || p.num_samples <= 0) return false;
  return tp_lds_bytes(a, p) <= 160 * 1024;
}

hipError_t mlp_tp_prepare(const FusedMlpArgs& a, const PersistArgs& p, PersistLaunch* out) {
  if (!mlp_tp_supported(a, p)) return hipErrorInvalidValue;
  const int ks = tp_ks(a.Din);
  const void* fn = a.ar.world > 1 ? pick_loss_tp<true>(a.loss_kind, ks) : pick_loss_tp<false>(a.loss_kind, ks);
  const size_t lds = tp_lds_bytes(a, p);
  if (lds > 64 * 1024) PTDT_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  out->fn = fn;
  out->threads = 64 * (a.H / 16);
  out->lds = lds;
  out->a = a;
  out->p = p;
  return hipSuccess;
}

}  // namespace ptdt
