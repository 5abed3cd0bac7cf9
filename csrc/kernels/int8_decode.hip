// LLM.int8 decode path (M <= 32 tokens) for gfx950: the same product as int8_mm.hip
// (bitsandbytes' outlier decomposition; reference BitsAndBytesConfig(load_in_8bit=True),
// NB03:52-56) in three launches and no host round trip:
//
//   i8_decode_stats  one workgroup per 512 input columns (64 chunks of 8), 4 row groups of <= 8
//                    rows: ONE round of 16-B loads; column absmax -> outlier bits (|x| > threshold)
//                    per chunk, the workgroup's outlier columns in column order, and per row the
//                    absmax over its non-outlier columns (a per-workgroup partial).
//   i8_decode_quant  same columns x Mp / 8 row-group workgroups: the row scales (max over the stats
//                    partials, fixed order) and x quantised to int8 (rint(x / s) with a true division,
//                    outlier columns 0, padding rows M..Mp-1 0), stored in the GEMV's MFMA operand
//                    order (1 KiB per 16-row tile and K step).
//   i8_decode_gemv   one workgroup per 16 output features, 4 or 8 waves splitting K: each lane streams
//                    16 weight bytes per 64-deep K step (plain loads -- non-temporal ones measured
//                    7-15 % slower -- 8 steps in flight) into v_mfma_i32_16x16x64_i8 against the
//                    quantised rows (L2-resident); with the pre-shuffled weights (i8_decode_pack) both
//                    operands of a step are one contiguous KiB per wave. Exact int32 partials meet in
//                    LDS in wave order; the epilogue dequantises and adds the outlier columns' fp32
//                    products (x[:, o] * q[n, o] * sw[n], in column order) and the bias.
//
// At decode shapes the product is a weight stream (Llama-7B MLP up-projection: 11008 x 4096
// int8 = 45 MB, 1 byte per weight where fp16 reads 2). Round 3 (separate outlier / quantise kernels,
// a host read of the outlier mask, a gathered fp32 matmul, the tiled int8 GEMM): 80 us at M = 16
// against 20 us for torch's fp16 GEMV; round 4: 17.3-18.0 us (profiles/r4_int8_decode_xq_ab.jsonl).
// Measured and dropped: the statistics and quantisation in ONE workgroup (12-36 us of dependent load
// rounds), quantising on the fly inside the GEMV (the work repeated in every workgroup: GEMV
// 16 -> 28 us), one launch with a cross-workgroup wait (12.4 us) or with every workgroup recomputing
// all column maxima (24 us).
#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

using i32x4 = __attribute__((ext_vector_type(4))) int;
constexpr int kStatChunks = 64;   // 8-column chunks per stats workgroup
constexpr int kListCap = 8 * kStatChunks;  // outlier columns a stats workgroup can list (all of them)
#ifndef PTDT_I8_WLOAD
#define PTDT_I8_WLOAD(p) (*(p))  // A/B: __builtin_nontemporal_load (GEMV 16.4 vs 15.3 us at 16 x 11008 x 4096)
#endif

template <typename T>
__device__ __forceinline__ float bits16_to_f32(uint16_t h) {
  if constexpr (std::is_same<T, _Float16>::value) return (float)__builtin_bit_cast(_Float16, h);
  else return bf16_to_f32(h);
}

// 8 consecutive elements (one 16-B load for 2-byte types, two for fp32) as floats
template <typename T>
__device__ __forceinline__ void load8(const T* p, float (&v)[8]) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    using u32x4 = __attribute__((ext_vector_type(4))) unsigned;
    const u32x4 u = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = bits16_to_f32<T>((uint16_t)(u[e >> 1] >> (16 * (e & 1))));
  }
}

// grid: ceil(nch / 64) workgroups of 256 threads; thread (row group rg = tid / 64, chunk c)
template <typename T>
__global__ void __launch_bounds__(256) i8_decode_stats_kernel(const T* __restrict__ x, int M, int K, float thr,
                                                              uint8_t* __restrict__ cbits, float* __restrict__ rowpart,
                                                              int* __restrict__ ocnt, int* __restrict__ olist) {
  __shared__ float cmax[4][kStatChunks][9];
  __shared__ uint8_t bits_l[kStatChunks];
  const int tid = threadIdx.x, lane = tid & 63, rg = tid >> 6;
  const int nch = K >> 3;
  const int c = blockIdx.x * kStatChunks + lane;
  const bool cv = c < nch;
  const int cc = cv ? c : nch - 1;
  const int m0 = 8 * rg;
  float v[8][8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int m = m0 + u < M ? m0 + u : M - 1;  // repeated rows do not change a max; masked below
    load8(x + (int64_t)m * K + 8 * cc, v[u]);
  }
  float a[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    a[e] = 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) a[e] = fmaxf(a[e], fabsf(v[u][e]));
    cmax[rg][lane][e] = m0 < M ? a[e] : 0.f;
  }
  __syncthreads();
  if (rg == 0) {
    uint32_t b = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float t = fmaxf(fmaxf(cmax[0][lane][e], cmax[1][lane][e]), fmaxf(cmax[2][lane][e], cmax[3][lane][e]));
      b |= (cv && t > thr ? 1u : 0u) << e;
    }
    bits_l[lane] = (uint8_t)b;
    if (cv) cbits[c] = (uint8_t)b;
    // this workgroup's outlier columns, column order
    const int cnt = __popc(b);
    int inc = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int t = __shfl_up(inc, d);
      if (lane >= d) inc += t;
    }
    int off = inc - cnt;
    for (int e = 0; e < 8; ++e)
      if (b & (1u << e)) olist[blockIdx.x * kListCap + off++] = 8 * c + e;
    if (lane == 63) ocnt[blockIdx.x] = inc;
  }
  __syncthreads();
  // per-row absmax over this workgroup's non-outlier columns
  const uint32_t ob = bits_l[lane];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    float r = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (cv && !(ob & (1u << e))) r = fmaxf(r, fabsf(v[u][e]));
    r = wave_max(r);
    if (lane == 0 && m0 + u < M) rowpart[blockIdx.x * 32 + m0 + u] = r;
  }
}

__device__ __forceinline__ float load_val(const void* p, int dtype, int64_t i) {
  if (dtype == kF32) return static_cast<const float*>(p)[i];
  if (dtype == kF16) return (float)static_cast<const _Float16*>(p)[i];
  return bf16_to_f32(static_cast<const uint16_t*>(p)[i]);
}
__device__ __forceinline__ void store_val(void* p, int dtype, int64_t i, float v) {
  if (dtype == kF32) static_cast<float*>(p)[i] = v;
  else if (dtype == kF16) static_cast<_Float16*>(p)[i] = (_Float16)v;
  else static_cast<uint16_t*>(p)[i] = f32_to_bf16(v);
}

// grid: (stats workgroups, Mp / 8 row groups). Row scales from the stats partials (all loads in one
// round), then this workgroup's 8-column chunks of its 8 rows quantised, 2 rows per thread (8 int8
// per store); workgroup (0, 0) publishes sx. The IEEE divisions are dependent instruction chains:
// spreading the rows over Mp / 8 times more workgroups shortens each wave's chain 4x.
template <typename T>
__global__ void __launch_bounds__(256) i8_decode_quant_kernel(const T* __restrict__ x, int M, int Mp, int K, int nsb,
                                                              const uint8_t* __restrict__ cbits,
                                                              const float* __restrict__ rowpart,
                                                              int8_t* __restrict__ xq, float* __restrict__ sx) {
  __shared__ float part[32 * 32];
  __shared__ float ssc[32];
  const int tid = threadIdx.x, lane = tid & 63, sub = tid >> 6;
  const int nch = K >> 3;
  const int c = blockIdx.x * kStatChunks + lane;
  const bool cv = c < nch;
  const int cc = cv ? c : nch - 1;
  const int m0 = 8 * blockIdx.y + 2 * sub;
  for (int i = tid; i < nsb * 32; i += 256) part[i] = rowpart[i];
  const uint32_t ob = cbits[cc];
  float v[2][8];
#pragma unroll
  for (int u = 0; u < 2; ++u) load8(x + (int64_t)(m0 + u < M ? m0 + u : M - 1) * K + 8 * cc, v[u]);
  __syncthreads();
  if (tid < 32) {
    float a = 0.f;
    for (int b = 0; b < nsb; ++b) a = fmaxf(a, part[b * 32 + tid]);  // exact: order-free
    const float sc = a > 0.f ? a / 127.f : 1.f;
    ssc[tid] = sc;
    if (blockIdx.x == 0 && blockIdx.y == 0 && tid < Mp) sx[tid] = tid < M ? sc : 1.f;
  }
  __syncthreads();
  if (!cv) return;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int m = m0 + u;
    if (m >= Mp) break;
    const float sc = ssc[m < M ? m : 0];  // x / s (IEEE division, as the reference), not x * (1 / s)
    uint32_t w[2] = {0u, 0u};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float q = (m < M && !(ob & (1u << e))) ? rintf(v[u][e] / sc) : 0.f;
      q = fminf(fmaxf(q, -127.f), 127.f);
      w[e >> 2] |= ((uint32_t)(int32_t)q & 0xffu) << (8 * (e & 3));
    }
    // MFMA operand order (as the packed weights): 16-row tile m / 16, K step, lane (m % 16, g), byte
    const int kk = 8 * c;
    const int64_t off = (((int64_t)(m >> 4) * (K >> 6) + (kk >> 6)) * 64 + ((kk & 63) >> 4) * 16 + (m & 15)) * 16 +
                        (kk & 15);
    *reinterpret_cast<uint2*>(xq + off) = make_uint2(w[0], w[1]);
  }
}

// MT: 16-row M tiles (Mp = 16 MT). K % 64 == 0. NWV waves split K (8 when there are too few
// 16-feature workgroups to fill the chip with 4). nsb: stats workgroups (outlier lists).
// PACKED: the weights come pre-shuffled (i8_decode_pack_kernel) -- each wave's load of one K step is
// one contiguous KiB -- instead of 16 rows x 64 B out of the row-major [N, K]; the outlier columns
// still read the row-major copy.
template <typename T, int MT, int NWV, bool PACKED>
__global__ void __launch_bounds__(64 * NWV) i8_decode_gemv_kernel(const T* __restrict__ x, const int8_t* __restrict__ xq,
                                                                  const float* __restrict__ sx,
                                                                  const int* __restrict__ ocnt,
                                                                  const int* __restrict__ olist, int nsb,
                                                                  const int8_t* __restrict__ W,
                                                                  const int8_t* __restrict__ Wp,
                                                                  const float* __restrict__ sw, const void* bias,
                                                                  int bias_dtype, void* y, int y_dtype, int M, int N,
                                                                  int K) {
  constexpr int U = 8;
  __shared__ i32x4 red[NWV - 1][MT][64];
  __shared__ int cnt_l[32];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  if (tid < nsb) cnt_l[tid] = ocnt[tid];  // visible after the reduction barrier below
  const int n = blockIdx.x * 16 + c;
  const int nr = n < N ? n : N - 1;  // edge rows load a real row, never store
  const int nk = K >> 6;
  const int s0 = (w * nk) / NWV, s1 = ((w + 1) * nk) / NWV;
  const int8_t* const wp = PACKED ? Wp + ((int64_t)blockIdx.x * nk * 64 + lane) * 16 : W + (int64_t)nr * K + 16 * g;
  const int8_t* xp[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) xp[i] = xq + ((int64_t)i * nk * 64 + lane) * 16;  // operand order: 1 KiB per step
  i32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = i32x4{0, 0, 0, 0};
  for (int s = s0; s < s1; s += U) {
    i32x4 b[U], a[U][MT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = (s + u < s1 ? s + u : s1 - 1) << 6;  // clamped tail re-reads a real step, unused
      b[u] = PTDT_I8_WLOAD(reinterpret_cast<const i32x4*>(wp + (PACKED ? (int64_t)k * 16 : (int64_t)k)));
#pragma unroll
      for (int i = 0; i < MT; ++i) a[u][i] = *reinterpret_cast<const i32x4*>(xp[i] + (int64_t)k * 16);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (s + u < s1)
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[i] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u][i], b[u], acc[i], 0, 0, 0);
  }
  if (w > 0)
#pragma unroll
    for (int i = 0; i < MT; ++i) red[w - 1][i][lane] = acc[i];
  __syncthreads();
  if (w != 0 || n >= N) return;
#pragma unroll
  for (int v = 0; v < NWV - 1; ++v)  // wave order: exact int32 sums
#pragma unroll
    for (int i = 0; i < MT; ++i) acc[i] += red[v][i][lane];
  const float swn = sw[n];
  const float bn = bias ? load_val(bias, bias_dtype, n) : 0.f;
  float o[MT][4];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) o[i][r] = 0.f;
  // outlier columns in column order (stats workgroups in order, each list in order):
  // x[m, col] * dequantised W[n, col]
  for (int b = 0; b < nsb; ++b) {
    const int no = cnt_l[b];
    for (int j = 0; j < no; ++j) {
      const int col = olist[b * kListCap + j];
      const float wq = (float)W[(int64_t)n * K + col] * swn;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 16 * i + 4 * g + r;
          o[i][r] += (m < M ? Cvt<T>::load(x, (int64_t)m * K + col) : 0.f) * wq;
        }
    }
  }
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 16 * i + 4 * g + r;
      if (m >= M) continue;
      float v = (float)acc[i][r] * sx[m] * swn;
      v += o[i][r];
      v += bn;
      store_val(y, y_dtype, (int64_t)m * N + n, v);
    }
}

// Pre-shuffle for the GEMV: Wp[tile][step][lane] = the 16 bytes lane (c, g) = (lane & 15, lane >> 4) of
// 16-feature tile `tile` loads at K step `step`: W[16 tile + c][64 step + 16 g ..] (rows past N repeat
// row N - 1, never stored). One thread per 16 B.
__global__ void __launch_bounds__(256) i8_decode_pack_kernel(const int8_t* __restrict__ W, int N, int K,
                                                             int8_t* __restrict__ Wp, int64_t chunks) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= chunks) return;
  const int nk = K >> 6;
  const int lane = (int)(i & 63);
  const int64_t blk = i >> 6;
  const int step = (int)(blk % nk);
  const int64_t tile = blk / nk;
  const int64_t n = min<int64_t>(tile * 16 + (lane & 15), N - 1);
  *reinterpret_cast<i32x4*>(Wp + i * 16) =
      *reinterpret_cast<const i32x4*>(W + n * K + 64 * step + 16 * (lane >> 4));
}

int stats_blocks(int K) { return ((K >> 3) + kStatChunks - 1) / kStatChunks; }

// workspace: xq [Mp][K] int8 | sx [32] f32 | cbits [K/8] (16-B padded) | rowpart [nsb][32] f32 | ocnt [nsb] |
// olist [nsb][kListCap]
struct Ws {
  int8_t* xq;
  float* sx;
  uint8_t* cbits;
  float* rowpart;
  int* ocnt;
  int* olist;
};
// byte offsets of the workspace pieces (all 16-B aligned: K % 64 == 0)
struct WsLayout {
  size_t sx, cbits, rowpart, ocnt, olist, total;
};
WsLayout ws_layout(int M, int K) {
  const size_t Mp = M <= 16 ? 16 : 32, nsb = (size_t)stats_blocks(K);
  WsLayout l;
  l.sx = Mp * (size_t)K;
  l.cbits = l.sx + 32 * sizeof(float);
  l.rowpart = l.cbits + ((size_t)(K >> 3) + 15) / 16 * 16;
  l.ocnt = l.rowpart + nsb * 32 * sizeof(float);
  l.olist = l.ocnt + nsb * sizeof(int);
  l.total = l.olist + nsb * kListCap * sizeof(int);
  return l;
}
Ws carve(void* base, int M, int K) {
  const WsLayout l = ws_layout(M, K);
  uint8_t* const b = static_cast<uint8_t*>(base);
  Ws w;
  w.xq = reinterpret_cast<int8_t*>(b);
  w.sx = reinterpret_cast<float*>(b + l.sx);
  w.cbits = b + l.cbits;
  w.rowpart = reinterpret_cast<float*>(b + l.rowpart);
  w.ocnt = reinterpret_cast<int*>(b + l.ocnt);
  w.olist = reinterpret_cast<int*>(b + l.olist);
  return w;
}

template <typename T>
hipError_t launch_t(const void* xv, int M, int K, float thr, const int8_t* W, const int8_t* Wp, const float* sw,
                    const void* bias, int bias_dtype, int N, void* y, int y_dtype, const Ws& ws, hipStream_t s) {
  const T* x = static_cast<const T*>(xv);
  const int nsb = stats_blocks(K), Mp = M <= 16 ? 16 : 32;
  hipLaunchKernelGGL(i8_decode_stats_kernel<T>, dim3(nsb), dim3(256), 0, s, x, M, K, thr, ws.cbits, ws.rowpart,
                     ws.ocnt, ws.olist);
  PTDT_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(i8_decode_quant_kernel<T>, dim3(nsb, Mp / 8), dim3(256), 0, s, x, M, Mp, K, nsb, ws.cbits,
                     ws.rowpart, ws.xq, ws.sx);
  PTDT_HIP_CHECK(hipGetLastError());
  const dim3 grid((unsigned)((N + 15) / 16));
  const bool wide = (N + 15) / 16 < 512;  // < 2 workgroups per CU: 8 waves each
#define PTDT_I8G(mt, nw, pk)                                                                                      \
  hipLaunchKernelGGL((i8_decode_gemv_kernel<T, mt, nw, pk>), grid, dim3(64 * nw), 0, s, x, ws.xq, ws.sx, ws.ocnt,      \
                     ws.olist, nsb, W, Wp, sw, bias, bias_dtype, y, y_dtype, M, N, K)
  if (Wp) {
    if (Mp == 16) {
      if (wide) PTDT_I8G(1, 8, true);
      else PTDT_I8G(1, 4, true);
    } else {
      if (wide) PTDT_I8G(2, 8, true);
      else PTDT_I8G(2, 4, true);
    }
  } else if (Mp == 16) {
    if (wide) PTDT_I8G(1, 8, false);
    else PTDT_I8G(1, 4, false);
  } else {
    if (wide) PTDT_I8G(2, 8, false);
    else PTDT_I8G(2, 4, false);
  }
#undef PTDT_I8G
  return hipGetLastError();
}

}  // namespace

size_t int8_decode_ws_bytes(int M, int K) { return ws_layout(M, K).total + 16; }

bool int8_decode_supported(int M, int N, int K) {
  return M >= 1 && M <= 32 && N >= 1 && K >= 64 && K % 64 == 0 && K <= kInt8DecodeMaxK;
}

size_t int8_decode_packed_bytes(int N, int K) { return (size_t)((N + 15) / 16) * 16 * (size_t)K; }

hipError_t int8_decode_pack(const int8_t* W, int N, int K, int8_t* Wp, hipStream_t s) {
  if (N < 1 || K < 64 || K % 64 != 0 || (reinterpret_cast<uintptr_t>(W) & 15) || (reinterpret_cast<uintptr_t>(Wp) & 15))
    return hipErrorInvalidValue;
  const int64_t chunks = (int64_t)int8_decode_packed_bytes(N, K) / 16;
  hipLaunchKernelGGL(i8_decode_pack_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, s, W, N, K, Wp, chunks);
  return hipGetLastError();
}

hipError_t int8_decode(const void* x, int x_dtype, int M, int K, float threshold, const int8_t* W, const int8_t* Wp,
                       const float* sw, const void* bias, int bias_dtype, int N, void* y, int y_dtype, void* ws,
                       hipStream_t s) {
  if (!int8_decode_supported(M, N, K)) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(W) & 15) || (reinterpret_cast<uintptr_t>(Wp) & 15) ||
      (reinterpret_cast<uintptr_t>(ws) & 15) ||
      (reinterpret_cast<uintptr_t>(x) & 15))
    return hipErrorInvalidValue;
  const Ws w = carve(ws, M, K);
  if (x_dtype == kF32)
    return launch_t<float>(x, M, K, threshold, W, Wp, sw, bias, bias_dtype, N, y, y_dtype, w, s);
  if (x_dtype == kF16) return launch_t<_Float16>(x, M, K, threshold, W, Wp, sw, bias, bias_dtype, N, y, y_dtype, w, s);
  return launch_t<uint16_t>(x, M, K, threshold, W, Wp, sw, bias, bias_dtype, N, y, y_dtype, w, s);
}

}  // namespace ptdt
