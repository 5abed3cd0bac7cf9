// Training-mode BatchNorm over channels-last activations with the ResNet
// epilogues fused: y = ReLU?(BN(x) + residual?), and its backward.
//
// Why (profiles/r1_resnet_window.md): in the ResNet-50 DDP step (bf16,
// channels_last, B=128) MIOpen's BatchNorm kernels plus the separate ReLU
// (clamp), residual add, ReLU-backward (threshold) and MIOpen's SubTensorOp
// passes take ~12 ms of a ~27 ms step -- all of it HBM-bound elementwise and
// reduction traffic over 11.1 M activations per image. Fusing the epilogues
// drops whole read/write passes; the reductions are written for the NHWC
// layout, where one activation row is C contiguous channels.
//
// Layout: x is [M, C] with unit channel stride (NHWC channels_last, M = N*H*W,
// or a plain [M, C] batch), bf16 or f32; weight/bias/statistics f32.
//
// Each pass loads 16 B per lane (8 bf16 / 4 f32 channels). A reduction launch is
// grid (row blocks, channel tiles): threads of a block cover TC channel vectors
// x RPI rows and walk the block's row range; partial sums are combined in LDS,
// written per row block, and the LAST row block of each channel tile to finish
// (atomic ticket; sc1 partial stores/loads, see last_block) reduces the partials
// in fixed order (deterministic), computes the per-channel coefficients and
// re-arms its ticket. So a BN forward is 2 launches (stats, apply) and a
// backward 2 launches (reduce, apply).
//
// Forward statistics use shifted sums (x - K, K = row 0 of the channel), so
// E[(x-K)^2] - E[x-K]^2 does not cancel catastrophically for |mean| >> std;
// the final combine runs in double. Running stats: torch's momentum update
// with the unbiased variance, num_batches_tracked incremented in-kernel.
//
// Backward (dy' = dy * [y > 0] with ReLU):
//   dbeta = sum dy',  dgamma = invstd * sum dy' (x - mean)
//   dx    = k dy' - k s2 (x - mean) - k s1,   k = gamma invstd,
//           s1 = dbeta / M, s2 = invstd^2 sum dy'(x - mean) / M
// i.e. dx = A dy' + B x + C per channel; with a residual branch d(residual) = dy'.
// An optional second addend dy2 (the residual gradient of the NEXT block, handed
// over by ops/norm.py's residual link) is summed into dy on the fly, replacing a
// separate add kernel (two reads + a write) by one extra read in each pass.
// The ReLU mask comes from the forward output y, or -- for BNs without a residual
// -- is recomputed from x with the forward's own fmaf(x, scale, shift), sparing
// one of the three reads in both backward passes.
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

constexpr int kThreads = 256;   // apply kernels
constexpr int kRed = 512;       // reduction kernels
constexpr int kRedBlocks = 384; // ~1.5 reduction blocks per CU
constexpr int kMaxGx = 256;     // row blocks per channel tile (bounds the last block's combine)

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return (e && e[0]) ? atoi(e) : dflt;
}
// channel vectors per block row of a reduction (a tile of TC*V channels): 32 (whole 512-B rows
// of a C = 256 bf16 tensor per 32 lanes) for tall tensors, where the wider tile measured up to
// 13 % faster, 8 below (more row blocks to fill the chip; profiles/r3_bn_sweep.md).
// PTDT_BN_TC forces one width.
constexpr int64_t kWideRows = 262144;
int forced_tc() {
  static const int v = [] {
    const int t = env_int("PTDT_BN_TC", 0);
    return (t == 4 || t == 8 || t == 16 || t == 32 || t == 64) ? t : 0;
  }();
  return v;
}
int max_tc(int64_t M) {
  const int f = forced_tc();
  return f ? f : (M >= kWideRows ? 32 : 8);
}
int min_tc() {  // the narrowest tile any M may get: sizes the ticket array
  const int f = forced_tc();
  return f ? f : 8;
}
// vectors per thread in flight in the elementwise passes (PTDT_BN_AU: 1, 2, 4)
int apply_unroll() {
  static const int v = [] {
    const int u = env_int("PTDT_BN_AU", 1);
    return (u == 1 || u == 2 || u == 4) ? u : 1;
  }();
  return v;
}
// cap on elementwise workgroups (grid-stride beyond it); PTDT_BN_APPLY_BLOCKS, 0 = uncapped
int apply_block_cap() {
  static const int v = env_int("PTDT_BN_APPLY_BLOCKS", 4096);
  return v;
}

template <typename T>
struct VecIO {
  static constexpr int V = 16 / sizeof(T);
  __device__ __forceinline__ static void load(const T* p, float (&v)[V]) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    if constexpr (sizeof(T) == 4) {
      v[0] = __uint_as_float(u.x); v[1] = __uint_as_float(u.y);
      v[2] = __uint_as_float(u.z); v[3] = __uint_as_float(u.w);
    } else {
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
      }
    }
  }
  __device__ __forceinline__ static void store(T* p, const float (&v)[V]) {
    uint4 u;
    if constexpr (sizeof(T) == 4) {
      u.x = __float_as_uint(v[0]); u.y = __float_as_uint(v[1]);
      u.z = __float_as_uint(v[2]); u.w = __float_as_uint(v[3]);
    } else {
      uint32_t w[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = pack_bf16x2(v[2 * i], v[2 * i + 1]);
      u.x = w[0]; u.y = w[1]; u.z = w[2]; u.w = w[3];
    }
    *reinterpret_cast<uint4*>(p) = u;
  }
};

// Row order of the reduction passes (PTDT_BN_INTERLEAVE=0: one contiguous slab per row block).
int interleave_rows() {
  static const int v = [] {
    const char* e = getenv("PTDT_BN_INTERLEAVE");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return v;
}

// reduction geometry knobs (profiles/r3_bn_sweep.md): minimum rows per thread (PTDT_BN_RPT) and the
// cap on reduction workgroups (PTDT_BN_RED_BLOCKS; the grid is at most cap / channel tiles row blocks)
int red_rows_per_thread() {
  static const int v = [] {
    const int r = env_int("PTDT_BN_RPT", 16);
    return r >= 1 && r <= 256 ? r : 16;
  }();
  return v;
}
int red_block_cap() {
  static const int v = [] {
    const int c = env_int("PTDT_BN_RED_BLOCKS", kRedBlocks);
    return c >= 64 && c <= 4096 ? c : kRedBlocks;
  }();
  return v;
}

struct Geom {
  int TC, RPI;       // channel vectors per row, rows per block iteration
  int gx, gy;        // row blocks, channel tiles
  int64_t rows_per_block;
};

template <typename T>
Geom geom(int64_t M, int C) {
  constexpr int V = VecIO<T>::V;
  Geom g;
  const int cv = C / V, mt = max_tc(M);
  g.TC = cv < mt ? cv : mt;
  g.RPI = kRed / g.TC;
  g.gy = (cv + g.TC - 1) / g.TC;
  const int rpt = red_rows_per_thread();
  int64_t want = (M + (int64_t)g.RPI * rpt - 1) / ((int64_t)g.RPI * rpt);  // >= rpt rows per thread
  int64_t cap = red_block_cap() / g.gy;
  if (cap > kMaxGx) cap = kMaxGx;
  if (cap < 1) cap = 1;
  g.gx = (int)(want < 1 ? 1 : (want > cap ? cap : want));
  g.rows_per_block = (M + g.gx - 1) / g.gx;
  g.gx = (int)((M + g.rows_per_block - 1) / g.rows_per_block);
  return g;
}

// Block-level combine of per-thread V-vectors over the RPI rows sharing a channel
// vector; returns (in threads t < TC*V) the block's sum for channel c0 + t.
template <int V, int NS>
__device__ __forceinline__ void block_rows_sum(float (&acc)[NS][V], float* sh, int TC, int RPI, float (&out)[NS]) {
  const int tid = threadIdx.x;
  const int width = TC * V;
  const int rr = tid / TC, tc = tid % TC;
  if (rr < RPI) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int v = 0; v < V; ++v) sh[(s * RPI + rr) * width + tc * V + v] = acc[s][v];
  }
  __syncthreads();
  if (tid < width) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      float a = 0.f;
      for (int r = 0; r < RPI; ++r) a += sh[(s * RPI + r) * width + tid];
      out[s] = a;
    }
  }
}

// Partials cross workgroups through sc1 (write-through, L1-bypassing) agent-scope relaxed stores and
// loads; the ticket's returned value names the last arriver (MI355X_MICROARCH.md, hand-off table row
// 1). The agent-scope release fence this replaced wrote back the XCD L2's dirty lines once per
// workgroup -- with the backward's g tensor streaming out through those L2s, a per-block cost at the
// tail of every reduction (profiles/r3_convbn.md shows the same fence at +110 us on a GEMM).
typedef __attribute__((address_space(1))) float gfloat_t;
// PTDT_BN_FENCE=1 (A/B measurements only): plain partial stores/loads behind the agent-scope
// release (every block) and acquire (last block) fences this hand-off replaced.
__device__ __forceinline__ void st_sc1(float* p, float v, bool fence = false) {
  if (fence) *p = v;
  else __hip_atomic_store((gfloat_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p, bool fence = false) {
  if (fence) return *p;
  return __hip_atomic_load((gfloat_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Last block of a channel tile: sum the gx row-block partials (two [gx][C] slabs) of the tile's
// `width` channels with ALL threads. Thread (part, quad) adds rows part, part + P, ... of 4
// consecutive channels (P = kRed / (width / 4) parts), kCombineRows rows x 2 slabs of two 8-B
// (agent-scope atomic) loads per 4 channels in flight per thread, so the whole combine is
// ceil(gx / (P kCombineRows)) round trips -- one for
// every ResNet-50 shape. (Round 4's form, one channel per thread and 4 rows in flight, took up to
// 32 dependent round trips on the wide layer-1 tiles: gx = 256 row blocks, 256 channels.) The P
// part-sums are then added in part order through LDS (deterministic). Result in threads t < width.
constexpr int kCombineRows = 4;
// 2 slabs x P x width doubles. P x width = 4 kRed for every tile width (P = 4 kRed / width), so this
// is the size every combine needs, not a worst case (ADVICE r5 asked to size it per launch). It does
// not cost occupancy: a CU holds 4 of these 512-thread blocks by waves (32), 128 KiB of LDS.
constexpr size_t kCombineLds = (size_t)2 * kRed * 4 * sizeof(double);
__device__ __forceinline__ void ld2_sc1(const float* p, float& x, float& y, bool fence) {
  uint64_t u;
  if (fence) u = *reinterpret_cast<const uint64_t*>(p);
  else u = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  x = __uint_as_float((uint32_t)u);
  y = __uint_as_float((uint32_t)(u >> 32));
}
__device__ __forceinline__ void combine_partials(const float* ws, int gx, int C, int cbase, int width, float* sh,
                                                 double& s0, double& s1, bool fence) {
  const int nq = width >> 2;
  const int P = kRed / nq;
  const int t = threadIdx.x, qd = t % nq, part = t / nq;
  const int c = cbase + 4 * qd;
  double a0[4] = {0.0, 0.0, 0.0, 0.0}, a1[4] = {0.0, 0.0, 0.0, 0.0};
  if (part < P && c < C) {
    const float* w0 = ws + c;
    const float* w1 = ws + (int64_t)gx * C + c;
    for (int b = part; b < gx; b += kCombineRows * P) {
      float u[kCombineRows][4], v[kCombineRows][4];
#pragma unroll
      for (int k = 0; k < kCombineRows; ++k) {
        const int r = b + k * P;
        if (r < gx) {
          ld2_sc1(w0 + (int64_t)r * C, u[k][0], u[k][1], fence);
          ld2_sc1(w0 + (int64_t)r * C + 2, u[k][2], u[k][3], fence);
          ld2_sc1(w1 + (int64_t)r * C, v[k][0], v[k][1], fence);
          ld2_sc1(w1 + (int64_t)r * C + 2, v[k][2], v[k][3], fence);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) u[k][i] = v[k][i] = 0.f;
        }
      }
#pragma unroll
      for (int k = 0; k < kCombineRows; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a0[i] += (double)u[k][i];
          a1[i] += (double)v[k][i];
        }
    }
  }
  __syncthreads();  // the reduction slots in sh are free again
  double* d = reinterpret_cast<double*>(sh);
  if (part < P) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      d[part * width + 4 * qd + i] = a0[i];
      d[(P + part) * width + 4 * qd + i] = a1[i];
    }
  }
  __syncthreads();
  s0 = s1 = 0.0;
  if (t < width) {
    for (int q = 0; q < P; ++q) {
      s0 += d[q * width + t];
      s1 += d[(P + q) * width + t];
    }
  }
}

// Atomic ticket: true in exactly one block per channel tile (the last to arrive), after every
// block's sc1 partial stores have landed (each wave drains its own, then the barrier), told by the
// value the relaxed agent-scope add returns. The flag travels through the kernel's one LDS array.
//
// Memory-model note (ISA-level, gfx950): the HIP/LLVM model gives relaxed atomics no
// happens-before, so correctness rests on the hardware, not the language: (1) the partials are
// written with sc1 stores (write-through to the coherent level) and each wave waits vmcnt(0)
// before the barrier, so they are globally visible before the ticket add issues; (2) the last
// block reads them with sc1 loads, which miss the non-coherent caches. The compiler cannot move
// those loads above the ticket: __syncthreads() after the flag write is a workgroup-scope
// release/acquire fence pair, and the explicit signal fence below pins the order in the IR too.
// tests/test_norm.py compares this hand-off with the fence-based one (PTDT_BN_FENCE=1) bit for bit
// on many-block shapes.
__device__ __forceinline__ bool last_block(int* ticket, int* sh_flag, bool fence) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (fence) {  // A/B: the replaced form (write-back of this XCD's L2 before the ticket)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const int prev = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == (int)gridDim.x - 1;
    if (last && fence) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *sh_flag = last;
  }
  __syncthreads();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);  // no load of the partials is hoisted above this point
  return *sh_flag != 0;
}

__device__ __forceinline__ void rearm(int* ticket) {
  __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename T>
__global__ void __launch_bounds__(kRed) bn_stats_kernel(const T* __restrict__ x, int64_t M, int C, int TC, int RPI,
                                                        int64_t rows_per_block, int il, float* ws, int* tickets,
                                                        BnParams p) {
  constexpr int V = VecIO<T>::V;
  constexpr int U = 8;  // rows in flight per thread
  extern __shared__ float sh[];  // 2 x RPI x TC*V reduction slots, then the last-block flag
  int* flag = reinterpret_cast<int*>(sh + 2 * kRed * V);
  const int tid = threadIdx.x, rr = tid / TC, tc = tid % TC;
  const int c0 = (blockIdx.y * TC + tc) * V;  // this thread's channels c0..c0+V
  const bool active = rr < RPI && c0 < C;
  // il bit 1: sweep the rows last to first (pass_dirs())
  const bool rev = (il & 2) != 0;
  il &= 1;
  auto row = [&](int64_t r) { return rev ? M - 1 - r : r; };
  // il: rows interleaved across the row blocks in RPI-row chunks (block b: chunks b, b + gx, ...),
  // so the grid sweeps the tensor front to back together, as the elementwise passes do; else each
  // block owns one contiguous slab of rows_per_block rows (gx separate streams)
  const int64_t rs = il ? (int64_t)gridDim.x * RPI : RPI;
  const int64_t rb = il ? (int64_t)blockIdx.x * RPI : (int64_t)blockIdx.x * rows_per_block;
  const int64_t re = il ? M : min(M, rb + rows_per_block);
  float acc[2][V];
#pragma unroll
  for (int v = 0; v < V; ++v) acc[0][v] = acc[1][v] = 0.f;
  if (active) {
    float K[V];
    VecIO<T>::load(x + c0, K);  // pivot: row 0 (same for every block)
    int64_t r = rb + rr;
    for (; r + (U - 1) * rs < re; r += U * rs) {  // U independent 16-B loads in flight
      float a[U][V];
#pragma unroll
      for (int u = 0; u < U; ++u) VecIO<T>::load(x + row(r + u * rs) * C + c0, a[u]);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int v = 0; v < V; ++v) {
          const float d = a[u][v] - K[v];
          acc[0][v] += d;
          acc[1][v] = fmaf(d, d, acc[1][v]);
        }
    }
    for (; r < re; r += rs) {
      float a[V];
      VecIO<T>::load(x + row(r) * C + c0, a);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float d = a[v] - K[v];
        acc[0][v] += d;
        acc[1][v] = fmaf(d, d, acc[1][v]);
      }
    }
  }
  float part[2];
  block_rows_sum<V, 2>(acc, sh, TC, RPI, part);
  const int width = TC * V;
  const int c = blockIdx.y * width + tid;
  if (tid < width && c < C) {
    st_sc1(ws + (int64_t)blockIdx.x * C + c, part[0], (p.fence_handoff != 0));
    st_sc1(ws + ((int64_t)gridDim.x + blockIdx.x) * C + c, part[1], (p.fence_handoff != 0));
  }
  if (!last_block(tickets + blockIdx.y, flag, (p.fence_handoff != 0))) return;
  double s, q;
  combine_partials(ws, (int)gridDim.x, C, blockIdx.y * width, width, sh, s, q, (p.fence_handoff != 0));
  if (tid < width && c < C) {
    const double Kc = (double)Cvt<T>::load(x, c);
    const double ms = s / (double)M;
    double var = q / (double)M - ms * ms;
    if (var < 0.0) var = 0.0;
    const double mean = Kc + ms;
    const float invstd = (float)(1.0 / sqrt(var + (double)p.eps));
    const float w = p.weight ? p.weight[c] : 1.f, b = p.bias ? p.bias[c] : 0.f;
    p.mean[c] = (float)mean;
    p.invstd[c] = invstd;
    p.scale[c] = w * invstd;
    p.shift[c] = b - (float)mean * w * invstd;
    if (p.running_mean) {
      const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
      p.running_mean[c] = (float)((1.0 - p.momentum) * p.running_mean[c] + p.momentum * mean);
      p.running_var[c] = (float)((1.0 - p.momentum) * p.running_var[c] + p.momentum * unbiased);
    }
  }
  if (tid == 0) {
    rearm(tickets + blockIdx.y);  // for the next launch (stream order)
    if (blockIdx.y == 0 && p.num_batches_tracked) *p.num_batches_tracked += 1;
  }
}

// MASKOUT: also write the ReLU mask, one byte per V-vector (bit v: y > 0), for a backward that
// then reads 1/16 (bf16) of a tensor instead of y
// Elementwise passes: each thread keeps AU vectors (stride apart) in flight per iteration.
template <typename T, bool RELU, bool RES, bool MASKOUT = false, int AU = 1>
__global__ void __launch_bounds__(kThreads) bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                            T* __restrict__ y, const float* __restrict__ scale,
                                                            const float* __restrict__ shift, int64_t nvec, int C,
                                                            int rev, uint8_t* __restrict__ mask) {
  constexpr int V = VecIO<T>::V;
  extern __shared__ float sh[];  // scale[C], shift[C]
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    sh[c] = scale[c];
    sh[C + c] = shift[c];
  }
  __syncthreads();
  const int cv = C / V;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  auto vid = [&](int64_t i) { return rev ? nvec - 1 - i : i; };  // rev: last vector first
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < nvec; i0 += AU * stride) {
    float a[AU][V], rv[AU][V];
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int64_t i = vid(i0 + u * stride);
      if (i0 + u * stride < nvec) {
        VecIO<T>::load(x + i * V, a[u]);
        if constexpr (RES) VecIO<T>::load(res + i * V, rv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      if (i0 + u * stride >= nvec) break;
      const int64_t i = vid(i0 + u * stride);
      const int c0 = (int)(i % cv) * V;
      unsigned bits = 0;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float o = fmaf(a[u][v], sh[c0 + v], sh[C + c0 + v]);
        if constexpr (RES) o += rv[u][v];
        if constexpr (RELU) o = fmaxf(o, 0.f);
        if constexpr (MASKOUT) bits |= (o > 0.f ? 1u : 0u) << v;
        a[u][v] = o;
      }
      VecIO<T>::store(y + i * V, a[u]);
      if constexpr (MASKOUT) mask[i] = (uint8_t)bits;
    }
  }
}

// MASK: 0 no ReLU, 1 ReLU mask from the forward output y, 2 ReLU mask recomputed
// from x (y > 0 <=> fmaf(x, scale, shift) > 0 bit-exactly, as the forward applied
// it): BNs without a residual skip reading y in both backward passes.
// MASK 3: the forward's bit mask (one byte per V-vector); `y` carries the bit as 0 / 1.
template <int MASK, int V>
__device__ __forceinline__ float masked_dy(float g, float x, float y, float sc, float sf) {
  if constexpr (MASK == 1 || MASK == 3) return y > 0.f ? g : 0.f;
  if constexpr (MASK == 2) return fmaf(x, sc, sf) > 0.f ? g : 0.f;
  return g;
}

// T-rounded value (what a T tensor holds): identity for f32
template <typename T>
__device__ __forceinline__ float round_to(float v) {
  if constexpr (sizeof(T) == 4) return v;
  return bf16_to_f32(f32_to_bf16(v));
}

// GOUT: the masked gradient g = mask (dy + dy2), rounded to T, is also written (to gout): it IS
// the residual gradient, and the apply pass then reads g and x only (bn_bwd_apply_g_kernel)
// instead of dy, dy2, x and the mask. The sums use the rounded g, so both passes agree.
template <typename T, int MASK, bool ADD2, bool GOUT = false>
__global__ void __launch_bounds__(kRed) bn_bwd_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                             const T* __restrict__ x,
                                                             const T* __restrict__ y, const uint8_t* __restrict__ mk,
                                                             T* __restrict__ gout, int64_t M, int C, int TC,
                                                             int RPI, int64_t rows_per_block, int il, float* ws,
                                                             int* tickets, BnBwdParams p) {
  constexpr int V = VecIO<T>::V;
  constexpr int U = 4;  // rows in flight per thread (x 2-3 loads each)
  extern __shared__ float sh[];
  int* flag = reinterpret_cast<int*>(sh + 2 * kRed * V);
  const int tid = threadIdx.x, rr = tid / TC, tc = tid % TC;
  const int c0 = (blockIdx.y * TC + tc) * V;
  const bool active = rr < RPI && c0 < C;
  const bool rev = (il & 2) != 0;
  il &= 1;
  auto row = [&](int64_t r) { return rev ? M - 1 - r : r; };
  const int64_t rs = il ? (int64_t)gridDim.x * RPI : RPI;  // row order: as in bn_stats_kernel
  const int64_t rb = il ? (int64_t)blockIdx.x * RPI : (int64_t)blockIdx.x * rows_per_block;
  const int64_t re = il ? M : min(M, rb + rows_per_block);
  float acc[2][V];
#pragma unroll
  for (int v = 0; v < V; ++v) acc[0][v] = acc[1][v] = 0.f;
  if (active) {
    float mu[V], sc[V], sf[V];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      mu[v] = p.mean[c0 + v];
      sc[v] = MASK == 2 ? p.scale[c0 + v] : 0.f;
      sf[v] = MASK == 2 ? p.shift[c0 + v] : 0.f;
    }
    int64_t r = rb + rr;
    const int cv = C / V;
    // ReLU mask operand o[v] (0 / 1 bits for MASK 3, y for MASK 1)
    auto load_mask = [&](int64_t row, int64_t off, float (&o)[V]) {
      if constexpr (MASK == 1) {
        VecIO<T>::load(y + off, o);
      } else if constexpr (MASK == 3) {
        const unsigned b = mk[row * cv + c0 / V];
#pragma unroll
        for (int v = 0; v < V; ++v) o[v] = (float)((b >> v) & 1u);
      }
    };
    auto finish = [&](float (&g)[V], const float (&a)[V], const float (&o)[V], int64_t off) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float gg = masked_dy<MASK, V>(g[v], a[v], (MASK == 1 || MASK == 3) ? o[v] : 0.f, sc[v], sf[v]);
        if constexpr (GOUT) gg = round_to<T>(gg);
        g[v] = gg;
        acc[0][v] += gg;
        acc[1][v] = fmaf(gg, a[v] - mu[v], acc[1][v]);
      }
      if constexpr (GOUT) VecIO<T>::store(gout + off, g);
    };
    for (; r + (U - 1) * rs < re; r += U * rs) {
      float g[U][V], a[U][V], o[U][V], g2[ADD2 ? U : 1][V];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t off = row(r + u * rs) * C + c0;
        VecIO<T>::load(dy + off, g[u]);
        if constexpr (ADD2) VecIO<T>::load(dy2 + off, g2[u]);
        VecIO<T>::load(x + off, a[u]);
        load_mask(row(r + u * rs), off, o[u]);
      }
      if constexpr (ADD2) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int v = 0; v < V; ++v) g[u][v] += g2[u][v];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) finish(g[u], a[u], o[u], row(r + u * rs) * C + c0);
    }
    for (; r < re; r += rs) {
      float g[V], a[V], o[V];
      const int64_t off = row(r) * C + c0;
      VecIO<T>::load(dy + off, g);
      if constexpr (ADD2) {
        float g2[V];
        VecIO<T>::load(dy2 + off, g2);
#pragma unroll
        for (int v = 0; v < V; ++v) g[v] += g2[v];
      }
      VecIO<T>::load(x + off, a);
      load_mask(row(r), off, o);
      finish(g, a, o, off);
    }
  }
  float part[2];
  block_rows_sum<V, 2>(acc, sh, TC, RPI, part);
  const int width = TC * V;
  const int c = blockIdx.y * width + tid;
  if (tid < width && c < C) {
    st_sc1(ws + (int64_t)blockIdx.x * C + c, part[0], (p.fence_handoff != 0));
    st_sc1(ws + ((int64_t)gridDim.x + blockIdx.x) * C + c, part[1], (p.fence_handoff != 0));
  }
  if (!last_block(tickets + blockIdx.y, flag, (p.fence_handoff != 0))) return;
  double sdy, sdx;
  combine_partials(ws, (int)gridDim.x, C, blockIdx.y * width, width, sh, sdy, sdx, (p.fence_handoff != 0));
  if (tid < width && c < C) {
    const double invstd = p.invstd[c], mean = p.mean[c];
    const double w = p.weight ? p.weight[c] : 1.0;
    if (p.dweight) p.dweight[c] = (float)(sdx * invstd);
    if (p.dbias) p.dbias[c] = (float)sdy;
    const double k = w * invstd, s1 = sdy / (double)M, s2 = invstd * invstd * sdx / (double)M;
    p.coef_a[c] = (float)k;
    p.coef_b[c] = (float)(-k * s2);
    p.coef_c[c] = (float)(k * s2 * mean - k * s1);
  }
  if (tid == 0) rearm(tickets + blockIdx.y);
}

// dx = A g + B x + C from the reduce pass's materialised g (GOUT): 2 reads + 1 write
template <typename T, int AU = 1>
__global__ void __launch_bounds__(kThreads) bn_bwd_apply_g_kernel(const T* __restrict__ g, const T* __restrict__ x,
                                                                  T* __restrict__ dx, BnBwdParams p, int64_t nvec,
                                                                  int C, int rev) {
  constexpr int V = VecIO<T>::V;
  extern __shared__ float sh[];  // A[C], B[C], C[C]
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    sh[c] = p.coef_a[c];
    sh[C + c] = p.coef_b[c];
    sh[2 * C + c] = p.coef_c[c];
  }
  __syncthreads();
  const int cv = C / V;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  auto vid = [&](int64_t i) { return rev ? nvec - 1 - i : i; };  // rev: last vector first
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < nvec; i0 += AU * stride) {
    float gg[AU][V], a[AU][V];
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int64_t i = vid(i0 + u * stride);
      if (i0 + u * stride < nvec) {
        VecIO<T>::load(g + i * V, gg[u]);
        VecIO<T>::load(x + i * V, a[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      if (i0 + u * stride >= nvec) break;
      const int64_t i = vid(i0 + u * stride);
      const int c0 = (int)(i % cv) * V;
#pragma unroll
      for (int v = 0; v < V; ++v)
        a[u][v] = fmaf(sh[c0 + v], gg[u][v], fmaf(sh[C + c0 + v], a[u][v], sh[2 * C + c0 + v]));
      VecIO<T>::store(dx + i * V, a[u]);
    }
  }
}

template <typename T, int MASK, bool RES, bool ADD2, int AU = 1>
__global__ void __launch_bounds__(kThreads) bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ dy2,
                                                                const T* __restrict__ x,
                                                                const T* __restrict__ y, T* __restrict__ dx,
                                                                T* __restrict__ dres, BnBwdParams p, int64_t nvec,
                                                                int C, int rev) {
  constexpr int V = VecIO<T>::V;
  extern __shared__ float sh[];  // A[C], B[C], C[C] (+ scale[C], shift[C] for MASK 2)
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    sh[c] = p.coef_a[c];
    sh[C + c] = p.coef_b[c];
    sh[2 * C + c] = p.coef_c[c];
    if constexpr (MASK == 2) {
      sh[3 * C + c] = p.scale[c];
      sh[4 * C + c] = p.shift[c];
    }
  }
  __syncthreads();
  const int cv = C / V;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  auto vid = [&](int64_t i) { return rev ? nvec - 1 - i : i; };  // rev: last vector first
  for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < nvec; i0 += AU * stride) {
    float g[AU][V], a[AU][V], o[AU][V], g2[ADD2 ? AU : 1][V];
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int64_t i = vid(i0 + u * stride);
      if (i0 + u * stride < nvec) {
        VecIO<T>::load(dy + i * V, g[u]);
        if constexpr (ADD2) VecIO<T>::load(dy2 + i * V, g2[u]);
        VecIO<T>::load(x + i * V, a[u]);
        if constexpr (MASK == 1) VecIO<T>::load(y + i * V, o[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      if (i0 + u * stride >= nvec) break;
      const int64_t i = vid(i0 + u * stride);
      const int c0 = (int)(i % cv) * V;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float gv = g[u][v];
        if constexpr (ADD2) gv += g2[u][v];
        gv = masked_dy<MASK, V>(gv, a[u][v], MASK == 1 ? o[u][v] : 0.f, MASK == 2 ? sh[3 * C + c0 + v] : 0.f,
                                MASK == 2 ? sh[4 * C + c0 + v] : 0.f);
        g[u][v] = gv;
        a[u][v] = fmaf(sh[c0 + v], gv, fmaf(sh[C + c0 + v], a[u][v], sh[2 * C + c0 + v]));
      }
      VecIO<T>::store(dx + i * V, a[u]);
      if constexpr (RES) VecIO<T>::store(dres + i * V, g[u]);
    }
  }
}

// LDS of a reduction launch: the row-sum slots (2 x kRed x V floats, then the last-block flag)
// and the combine's part sums (kCombineLds) share one array
template <typename T>
size_t red_lds() {
  const size_t rows = (size_t)2 * kRed * VecIO<T>::V * sizeof(float) + 16;
  return rows > kCombineLds ? rows : kCombineLds;
}

int apply_grid(int64_t nvec) {
  const int au = apply_unroll(), cap = apply_block_cap();
  int64_t per = (int64_t)kThreads * (cap > 0 ? 4 : au);  // >= 4 vectors per thread when capped
  int64_t b = (nvec + per - 1) / per;
  if (cap > 0 && b > cap) b = cap;
  return (int)(b < 1 ? 1 : b);
}

// Sweep direction of each pass (PTDT_BN_DIR bits: 1 stats, 2 forward apply, 4 backward reduce,
// 8 backward apply; set = last row first). Consecutive passes over one tensor in opposite
// directions re-read the most recently touched lines first, which the 256 MiB Infinity Cache
// still holds (MI355X_MICROARCH.md "Infinity Cache").
int pass_dirs() {
  static const int v = env_int("PTDT_BN_DIR", 0);
  return v;
}
int dir(int bit) { return (pass_dirs() & bit) ? 1 : 0; }

// runtime AU -> template
template <typename F>
hipError_t with_au(F&& f) {
  switch (apply_unroll()) {
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    default: f(std::integral_constant<int, 1>{}); break;
  }
  return hipGetLastError();
}

template <typename T>
hipError_t fwd_impl(const BnFwdArgs& a, hipStream_t s) {
  constexpr int V = VecIO<T>::V;
  if (a.C % V != 0) return hipErrorInvalidValue;
  const Geom g = geom<T>(a.M, a.C);
  const size_t sh_red = red_lds<T>();
  if (!a.stats_ready) {
    hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(g.gx, g.gy), dim3(kRed), sh_red, s, static_cast<const T*>(a.x),
                       a.M, a.C, g.TC, g.RPI, g.rows_per_block, interleave_rows() | (dir(1) << 1), a.workspace,
                       a.tickets, a.p);
    PTDT_HIP_CHECK(hipGetLastError());
  }
  if (a.y == nullptr) return hipSuccess;  // statistics only (the apply runs in the consumer, e.g. a pool)
  const int64_t nvec = a.M * a.C / V;
  const size_t sh_ap = (size_t)2 * a.C * sizeof(float);
  const T* x = static_cast<const T*>(a.x);
  const T* r = static_cast<const T*>(a.residual);
  T* y = static_cast<T*>(a.y);
  const dim3 grid(apply_grid(nvec)), blk(kThreads);
  const float *sc = a.p.scale, *sf = a.p.shift;
  uint8_t* mo = a.mask_out;
  const int C = a.C;
  return with_au([&](auto au) {
    constexpr int AU = decltype(au)::value;
    if (a.relu) {
      if (r && mo) hipLaunchKernelGGL((bn_apply_kernel<T, true, true, true, AU>), grid, blk, sh_ap, s, x, r, y, sc, sf, nvec, C, dir(2), mo);
      else if (r) hipLaunchKernelGGL((bn_apply_kernel<T, true, true, false, AU>), grid, blk, sh_ap, s, x, r, y, sc, sf, nvec, C, dir(2), nullptr);
      else hipLaunchKernelGGL((bn_apply_kernel<T, true, false, false, AU>), grid, blk, sh_ap, s, x, r, y, sc, sf, nvec, C, dir(2), nullptr);
    } else {
      if (r) hipLaunchKernelGGL((bn_apply_kernel<T, false, true, false, AU>), grid, blk, sh_ap, s, x, r, y, sc, sf, nvec, C, dir(2), nullptr);
      else hipLaunchKernelGGL((bn_apply_kernel<T, false, false, false, AU>), grid, blk, sh_ap, s, x, r, y, sc, sf, nvec, C, dir(2), nullptr);
    }
  });
}

template <typename T>
hipError_t apply_impl(const void* x, const void* res, void* y, const float* scale, const float* shift, int64_t M,
                      int C, int relu, hipStream_t s) {
  constexpr int V = VecIO<T>::V;
  if (C % V != 0) return hipErrorInvalidValue;
  const int64_t nvec = M * C / V;
  const size_t sh_ap = (size_t)2 * C * sizeof(float);
  const T* xx = static_cast<const T*>(x);
  const T* r = static_cast<const T*>(res);
  T* yy = static_cast<T*>(y);
  const dim3 grid(apply_grid(nvec)), blk(kThreads);
  return with_au([&](auto au) {
    constexpr int AU = decltype(au)::value;
    if (relu) {
      if (r) hipLaunchKernelGGL((bn_apply_kernel<T, true, true, false, AU>), grid, blk, sh_ap, s, xx, r, yy, scale, shift, nvec, C, 0, nullptr);
      else hipLaunchKernelGGL((bn_apply_kernel<T, true, false, false, AU>), grid, blk, sh_ap, s, xx, r, yy, scale, shift, nvec, C, 0, nullptr);
    } else {
      if (r) hipLaunchKernelGGL((bn_apply_kernel<T, false, true, false, AU>), grid, blk, sh_ap, s, xx, r, yy, scale, shift, nvec, C, 0, nullptr);
      else hipLaunchKernelGGL((bn_apply_kernel<T, false, false, false, AU>), grid, blk, sh_ap, s, xx, r, yy, scale, shift, nvec, C, 0, nullptr);
    }
  });
}

template <typename T, int MASK, bool ADD2>
hipError_t bwd_launch(const BnBwdArgs& a, const Geom& g, hipStream_t s) {
  constexpr int V = VecIO<T>::V;
  const size_t sh_red = red_lds<T>();
  const T* dy = static_cast<const T*>(a.dy);
  const T* dy2 = static_cast<const T*>(a.dy2);
  const T* x = static_cast<const T*>(a.x);
  const T* y = static_cast<const T*>(a.y);
  const int64_t nvec = a.M * a.C / V;
  T* dx = static_cast<T*>(a.dx);
  T* dr = static_cast<T*>(a.dres);
  const dim3 grid(apply_grid(nvec)), blk(kThreads);
  if (a.reduce_only) {  // g materialised for a consumer that applies the coefficients itself
    if (!dr) return hipErrorInvalidValue;
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, MASK, ADD2, true>), dim3(g.gx, g.gy), dim3(kRed), sh_red, s, dy, dy2,
                       x, y, a.mask, dr, a.M, a.C, g.TC, g.RPI, g.rows_per_block, interleave_rows() | (dir(4) << 1),
                       a.workspace, a.tickets, a.p);
    return hipGetLastError();
  }
  if (dr) {  // the residual gradient is wanted: the reduce pass writes g there, the apply reads g and x
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, MASK, ADD2, true>), dim3(g.gx, g.gy), dim3(kRed), sh_red, s, dy, dy2,
                       x, y, a.mask, dr, a.M, a.C, g.TC, g.RPI, g.rows_per_block, interleave_rows() | (dir(4) << 1), a.workspace,
                       a.tickets, a.p);
    PTDT_HIP_CHECK(hipGetLastError());
    return with_au([&](auto au) {
      hipLaunchKernelGGL((bn_bwd_apply_g_kernel<T, decltype(au)::value>), grid, blk, (size_t)3 * a.C * sizeof(float),
                         s, static_cast<const T*>(dr), x, dx, a.p, nvec, a.C, dir(8));
    });
  }
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, MASK, ADD2>), dim3(g.gx, g.gy), dim3(kRed), sh_red, s, dy, dy2, x, y,
                     a.mask, nullptr, a.M, a.C, g.TC, g.RPI, g.rows_per_block, interleave_rows() | (dir(4) << 1), a.workspace,
                     a.tickets, a.p);
  PTDT_HIP_CHECK(hipGetLastError());
  if constexpr (MASK == 3) {
    return hipErrorInvalidValue;  // bit masks come with a residual (RES): the g path above
  } else {
    const size_t sh_ap = (size_t)(MASK == 2 ? 5 : 3) * a.C * sizeof(float);
    return with_au([&](auto au) {
      hipLaunchKernelGGL((bn_bwd_apply_kernel<T, MASK, false, ADD2, decltype(au)::value>), grid, blk, sh_ap, s, dy,
                         dy2, x, y, dx, dr, a.p, nvec, a.C, dir(8));
    });
  }
}

template <typename T, int MASK>
hipError_t bwd_launch2(const BnBwdArgs& a, const Geom& g, hipStream_t s) {
  return a.dy2 != nullptr ? bwd_launch<T, MASK, true>(a, g, s) : bwd_launch<T, MASK, false>(a, g, s);
}

template <typename T>
hipError_t bwd_impl(const BnBwdArgs& a, hipStream_t s) {
  constexpr int V = VecIO<T>::V;
  if (a.C % V != 0) return hipErrorInvalidValue;
  const Geom g = geom<T>(a.M, a.C);
  if (!a.relu) return bwd_launch2<T, 0>(a, g, s);
  if (a.mask != nullptr) {
    if (a.dres == nullptr) return hipErrorInvalidValue;
    return bwd_launch2<T, 3>(a, g, s);
  }
  if (a.y != nullptr) return bwd_launch2<T, 1>(a, g, s);
  if (a.p.scale == nullptr || a.p.shift == nullptr) return hipErrorInvalidValue;
  return bwd_launch2<T, 2>(a, g, s);
}

}  // namespace

int64_t bn_workspace_floats(int64_t M, int C, int dtype) {
  const Geom g = dtype == kF32 ? geom<float>(M, C) : geom<uint16_t>(M, C);
  return (int64_t)2 * g.gx * C;
}
int bn_num_tickets(int C, int dtype) {
  const int V = dtype == kF32 ? 4 : 8;
  const int cv = C / V, mt = min_tc();
  const int TC = cv < mt ? cv : mt;
  return (cv + TC - 1) / TC;
}

// PTDT_BN_FENCE=1: the fence-based partial hand-off, for same-box A/B measurements only
int fence_handoff() {
  static const int v = env_int("PTDT_BN_FENCE", 0) != 0;
  return v;
}

hipError_t bn_forward_train(const BnFwdArgs& a0, hipStream_t s) {
  if (a0.M <= 0 || a0.C <= 0) return hipErrorInvalidValue;
  BnFwdArgs a = a0;
  a.p.fence_handoff = fence_handoff();
  return a.dtype == kF32 ? fwd_impl<float>(a, s) : fwd_impl<uint16_t>(a, s);
}

hipError_t bn_apply(const void* x, const void* residual, void* y, int dtype, const float* scale, const float* shift,
                    int64_t M, int C, int relu, hipStream_t s) {
  if (M <= 0 || C <= 0) return hipErrorInvalidValue;
  return dtype == kF32 ? apply_impl<float>(x, residual, y, scale, shift, M, C, relu, s)
                       : apply_impl<uint16_t>(x, residual, y, scale, shift, M, C, relu, s);
}

hipError_t bn_backward(const BnBwdArgs& a0, hipStream_t s) {
  if (a0.M <= 0 || a0.C <= 0) return hipErrorInvalidValue;
  BnBwdArgs a = a0;
  a.p.fence_handoff = fence_handoff();
  return a.dtype == kF32 ? bwd_impl<float>(a, s) : bwd_impl<uint16_t>(a, s);
}

}  // namespace ptdt
