// LLM.int8 decode path (M <= 32 tokens) for gfx950: the same product as int8_mm.hip
// (bitsandbytes' outlier decomposition; reference BitsAndBytesConfig(load_in_8bit=True),
// NB03:52-56) in TWO launches and no host round trip:
//
//   i8_decode_prep  (one workgroup): column absmax over the M rows -> outlier columns
//                   (|x| > threshold), compacted IN COLUMN ORDER into a device list;
//                   per-row absmax over the other columns, x quantised to int8 (outlier
//                   columns 0, rows M..Mp-1 0), the outlier columns' values kept in fp32.
//   i8_decode_gemv  one workgroup per 16 output features: 4 (8 at N < 8192) waves split K, each streams
//                   its quarter of the 16 weight rows (non-temporal 16-B loads, 8 K-steps
//                   in flight) into v_mfma_i32_16x16x64_i8 against the quantised rows
//                   (L2-resident), exact int32 partials meet in LDS in wave order, and the
//                   epilogue dequantises and adds the outlier columns' fp32 products
//                   (x[:, o] * q[n, o] * sw[n], in list order) and the bias.
//
// At decode shapes the product is a weight stream (Llama-7B MLP up-projection: 11008 x 4096
// int8 = 45 MB, 1 byte per weight where fp16 reads 2): the round-3 path (separate outlier /
// quantise kernels, a host read of the outlier mask, a gathered fp32 matmul, the tiled int8
// GEMM) took 80 us at M = 16 against 21 us for torch's fp16 GEMV.
#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

using i32x4 = __attribute__((ext_vector_type(4))) int;
constexpr int kPrep = 1024;

// 8 consecutive elements (one 16-B load for 2-byte types, two for fp32) as floats
template <typename T>
__device__ __forceinline__ void load8(const T* p, float (&v)[8]) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const T* h = reinterpret_cast<const T*>(&u);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = Cvt<T>::load(h, e);
  }
}

// One workgroup; every global read is a 16-B chunk of 8 columns with up to 8 chunks in flight per
// thread (round 4's first version looped over rows with one dependent 2-byte load per iteration:
// ~60 us of load latency at M = 32).
//   pass 1: thread t owns column chunks t, t + kPrep: column absmax over the M rows, outlier bits
//           per chunk (LDS), outlier columns compacted in column order (block scan of the counts)
//   pass 2: one wave per row: absmax over the non-outlier columns, quantise (8 int8 per store), the
//           outlier columns' values kept in fp32; padding rows M..Mp-1 zero
template <typename T>
__global__ void __launch_bounds__(kPrep) i8_decode_prep_kernel(const T* __restrict__ x, int M, int Mp, int K, float thr,
                                                               int8_t* __restrict__ xq, float* __restrict__ sx,
                                                               int* __restrict__ oidx, int* __restrict__ ocnt,
                                                               float* __restrict__ xo) {
  __shared__ uint8_t cbits[kInt8DecodeMaxK / 8];
  __shared__ int wcnt[kPrep / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nch = K >> 3;
  // ---- pass 1
  int base = 0;
  for (int c0 = 0; c0 < nch; c0 += kPrep) {
    const int c = c0 + tid;
    uint32_t bits = 0;
    if (c < nch) {
      float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int m0 = 0; m0 < M; m0 += 8) {
        float v[8][8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int m = m0 + u < M ? m0 + u : M - 1;  // a repeated row does not change the max
          load8(x + (int64_t)m * K + 8 * c, v[u]);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
          for (int e = 0; e < 8; ++e) a[e] = fmaxf(a[e], fabsf(v[u][e]));
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) bits |= (a[e] > thr ? 1u : 0u) << e;
      cbits[c] = (uint8_t)bits;
    }
    // exclusive scan of the per-thread counts in thread (= column) order
    const int cnt = __popc(bits);
    int inc = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int t = __shfl_up(inc, d);
      if (lane >= d) inc += t;
    }
    if (lane == 63) wcnt[wid] = inc;
    __syncthreads();
    int off = base + inc - cnt, tot = 0;
    for (int v = 0; v < kPrep / 64; ++v) {
      if (v < wid) off += wcnt[v];
      tot += wcnt[v];
    }
    for (int e = 0; e < 8; ++e)
      if (bits & (1u << e)) oidx[off++] = 8 * c + e;
    base += tot;
    __syncthreads();  // wcnt reused by the next round; cbits complete for pass 2
  }
  if (tid == 0) *ocnt = base;
  // ---- pass 2
  constexpr int J = 8;  // chunks per lane in flight
  for (int m = wid; m < Mp; m += kPrep / 64) {
    int8_t* const qr = xq + (int64_t)m * K;
    if (m >= M) {
      for (int c = lane; c < nch; c += 64) *reinterpret_cast<uint2*>(qr + 8 * c) = make_uint2(0u, 0u);
      for (int j = lane; j < base; j += 64) xo[(int64_t)j * Mp + m] = 0.f;
      if (lane == 0) sx[m] = 1.f;
      continue;
    }
    const T* const xr = x + (int64_t)m * K;
    float a = 0.f;
    for (int cb = 0; cb < nch; cb += 64 * J) {
      float v[J][8];
#pragma unroll
      for (int u = 0; u < J; ++u) {
        const int c = cb + 64 * u + lane;
        load8(xr + 8 * (c < nch ? c : nch - 1), v[u]);
      }
#pragma unroll
      for (int u = 0; u < J; ++u) {
        const int c = cb + 64 * u + lane;
        const uint32_t ob = c < nch ? cbits[c] : 0xffu;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (!(ob & (1u << e))) a = fmaxf(a, fabsf(v[u][e]));
      }
    }
    a = wave_max(a);
    const float sc = a > 0.f ? a / 127.f : 1.f;
    const float inv = 1.f / sc;
    for (int cb = 0; cb < nch; cb += 64 * J) {
      float v[J][8];
#pragma unroll
      for (int u = 0; u < J; ++u) {
        const int c = cb + 64 * u + lane;
        load8(xr + 8 * (c < nch ? c : nch - 1), v[u]);
      }
#pragma unroll
      for (int u = 0; u < J; ++u) {
        const int c = cb + 64 * u + lane;
        if (c >= nch) continue;
        const uint32_t ob = cbits[c];
        uint32_t w[2] = {0u, 0u};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float q = (ob & (1u << e)) ? 0.f : rintf(v[u][e] * inv);
          q = fminf(fmaxf(q, -127.f), 127.f);
          w[e >> 2] |= ((uint32_t)(int32_t)q & 0xffu) << (8 * (e & 3));
        }
        *reinterpret_cast<uint2*>(qr + 8 * c) = make_uint2(w[0], w[1]);
      }
    }
    for (int j = lane; j < base; j += 64) xo[(int64_t)j * Mp + m] = Cvt<T>::load(xr, oidx[j]);
    if (lane == 0) sx[m] = sc;
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

// MT: 16-row M tiles (Mp = 16 MT). K % 64 == 0. NWV waves split K (8 when there are too few
// 16-feature workgroups to fill the chip with 4).
template <int MT, int NWV>
__global__ void __launch_bounds__(64 * NWV) i8_decode_gemv_kernel(const int8_t* __restrict__ xq,
                                                               const float* __restrict__ sx,
                                                               const int8_t* __restrict__ W,
                                                               const float* __restrict__ sw,
                                                               const int* __restrict__ oidx,
                                                               const int* __restrict__ ocnt,
                                                               const float* __restrict__ xo, const void* bias,
                                                               int bias_dtype, void* y, int y_dtype, int M, int N,
                                                               int K) {
  constexpr int Mp = 16 * MT, U = 8;
  __shared__ i32x4 red[NWV - 1][MT][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int n = blockIdx.x * 16 + c;
  const int nr = n < N ? n : N - 1;  // edge rows load a real row, never store
  const int nk = K >> 6;
  const int s0 = (w * nk) / NWV, s1 = ((w + 1) * nk) / NWV;
  const int8_t* const wp = W + (int64_t)nr * K + 16 * g;
  const int8_t* xp[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) xp[i] = xq + (int64_t)(16 * i + c) * K + 16 * g;
  i32x4 acc[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i] = i32x4{0, 0, 0, 0};
  for (int s = s0; s < s1; s += U) {
    i32x4 b[U], a[U][MT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = (s + u < s1 ? s + u : s1 - 1) << 6;  // clamped tail re-reads a real step, unused
      b[u] = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(wp + k));
#pragma unroll
      for (int i = 0; i < MT; ++i) a[u][i] = *reinterpret_cast<const i32x4*>(xp[i] + k);
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
  const int no = *ocnt;
  float o[MT][4];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) o[i][r] = 0.f;
  for (int j = 0; j < no; ++j) {  // outlier columns, list order: x[m, col] * dequantised W[n, col]
    const float wq = (float)W[(int64_t)n * K + oidx[j]] * swn;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[i][r] += xo[(int64_t)j * Mp + 16 * i + 4 * g + r] * wq;
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

template <typename T>
hipError_t prep_t(const void* x, int M, int Mp, int K, float thr, int8_t* xq, float* sx, int* oidx, int* ocnt,
                  float* xo, hipStream_t s) {
  hipLaunchKernelGGL(i8_decode_prep_kernel<T>, dim3(1), dim3(kPrep), 0, s, static_cast<const T*>(x), M, Mp, K, thr, xq,
                     sx, oidx, ocnt, xo);
  return hipGetLastError();
}

}  // namespace

size_t int8_decode_ws_bytes(int M, int K) {
  const int Mp = M <= 16 ? 16 : 32;
  return (size_t)Mp * K + 4 * (size_t)Mp + 4 * (size_t)K + 16 + 4 * (size_t)K * Mp;
}

bool int8_decode_supported(int M, int N, int K) {
  return M >= 1 && M <= 32 && N >= 1 && K >= 64 && K % 64 == 0 && K <= kInt8DecodeMaxK;
}

hipError_t int8_decode(const void* x, int x_dtype, int M, int K, float threshold, const int8_t* W, const float* sw,
                       const void* bias, int bias_dtype, int N, void* y, int y_dtype, void* ws, hipStream_t s) {
  if (!int8_decode_supported(M, N, K)) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(W) & 15) || (reinterpret_cast<uintptr_t>(ws) & 15) ||
      (reinterpret_cast<uintptr_t>(x) & 15))
    return hipErrorInvalidValue;
  const int Mp = M <= 16 ? 16 : 32;
  int8_t* xq = static_cast<int8_t*>(ws);
  float* sx = reinterpret_cast<float*>(xq + (size_t)Mp * K);
  int* oidx = reinterpret_cast<int*>(sx + Mp);
  int* ocnt = oidx + K;
  float* xo = reinterpret_cast<float*>(ocnt + 4);
  hipError_t e = x_dtype == kF32   ? prep_t<float>(x, M, Mp, K, threshold, xq, sx, oidx, ocnt, xo, s)
                 : x_dtype == kF16 ? prep_t<_Float16>(x, M, Mp, K, threshold, xq, sx, oidx, ocnt, xo, s)
                                   : prep_t<uint16_t>(x, M, Mp, K, threshold, xq, sx, oidx, ocnt, xo, s);
  if (e != hipSuccess) return e;
  const dim3 grid((unsigned)((N + 15) / 16));
  const bool wide = (N + 15) / 16 < 512;  // < 2 workgroups per CU: 8 waves each
#define PTDT_I8G(mt, nw)                                                                                     \
  hipLaunchKernelGGL((i8_decode_gemv_kernel<mt, nw>), grid, dim3(64 * nw), 0, s, xq, sx, W, sw, oidx, ocnt, xo, \
                     bias, bias_dtype, y, y_dtype, M, N, K)
  if (Mp == 16) {
    if (wide) PTDT_I8G(1, 8);
    else PTDT_I8G(1, 4);
  } else {
    if (wide) PTDT_I8G(2, 8);
    else PTDT_I8G(2, 4);
  }
#undef PTDT_I8G
  return hipGetLastError();
}

}  // namespace ptdt
