// LLM.int8 decode path (M <= 32 tokens) for gfx950: the same product as int8_mm.hip
// (bitsandbytes' outlier decomposition; reference BitsAndBytesConfig(load_in_8bit=True),
// NB03:52-56) in TWO launches and no host round trip:
//
//   i8_decode_prep  (one workgroup): column absmax over the M rows -> outlier columns
//                   (|x| > threshold), compacted IN COLUMN ORDER into a device list;
//                   per-row absmax over the other columns, x quantised to int8 (outlier
//                   columns 0, rows M..Mp-1 0), the outlier columns' values kept in fp32.
//   i8_decode_gemv  one workgroup per 16 output features: 4 waves split K, each streams
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
constexpr int kGemv = 256;

template <typename T>
__global__ void __launch_bounds__(kPrep) i8_decode_prep_kernel(const T* __restrict__ x, int M, int Mp, int K, float thr,
                                                               int8_t* __restrict__ xq, float* __restrict__ sx,
                                                               int* __restrict__ oidx, int* __restrict__ ocnt,
                                                               float* __restrict__ xo) {
  __shared__ uint8_t omask[kInt8DecodeMaxK];
  __shared__ int wcnt[kPrep / 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // ---- pass 1 (column-parallel): outlier flags, compacted in column order
  int base = 0;
  for (int kc = 0; kc < K; kc += kPrep) {
    const int k = kc + tid;
    bool out = false;
    if (k < K) {
      float a = 0.f;
      for (int m = 0; m < M; ++m) a = fmaxf(a, fabsf(Cvt<T>::load(x, (int64_t)m * K + k)));
      out = a > thr;
      omask[k] = out ? 1 : 0;
    }
    const uint64_t bal = __ballot(out);
    if (lane == 0) wcnt[wid] = __popcll(bal);
    __syncthreads();
    int off = base, tot = 0;
    for (int v = 0; v < kPrep / 64; ++v) {
      if (v < wid) off += wcnt[v];
      tot += wcnt[v];
    }
    if (out) oidx[off + __popcll(bal & ((1ull << lane) - 1ull))] = k;
    base += tot;
    __syncthreads();  // wcnt reused by the next chunk
  }
  if (tid == 0) *ocnt = base;
  // ---- pass 2 (one wave per row): absmax over the non-outlier columns, quantise, outlier values
  for (int m = wid; m < Mp; m += kPrep / 64) {
    if (m >= M) {
      for (int k = lane; k < K; k += 64) xq[(int64_t)m * K + k] = 0;
      for (int j = lane; j < base; j += 64) xo[(int64_t)j * Mp + m] = 0.f;
      if (lane == 0) sx[m] = 1.f;
      continue;
    }
    const T* xr = x + (int64_t)m * K;
    float a = 0.f;
    for (int k = lane; k < K; k += 64)
      if (!omask[k]) a = fmaxf(a, fabsf(Cvt<T>::load(xr, k)));
    a = wave_max(a);
    const float sc = a > 0.f ? a / 127.f : 1.f;
    const float inv = 1.f / sc;
    for (int k = lane; k < K; k += 64) {
      float v = omask[k] ? 0.f : rintf(Cvt<T>::load(xr, k) * inv);
      v = fminf(fmaxf(v, -127.f), 127.f);
      xq[(int64_t)m * K + k] = (int8_t)v;
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

// MT: 16-row M tiles (Mp = 16 MT). K % 64 == 0.
template <int MT>
__global__ void __launch_bounds__(kGemv) i8_decode_gemv_kernel(const int8_t* __restrict__ xq,
                                                               const float* __restrict__ sx,
                                                               const int8_t* __restrict__ W,
                                                               const float* __restrict__ sw,
                                                               const int* __restrict__ oidx,
                                                               const int* __restrict__ ocnt,
                                                               const float* __restrict__ xo, const void* bias,
                                                               int bias_dtype, void* y, int y_dtype, int M, int N,
                                                               int K) {
  constexpr int Mp = 16 * MT, U = 8;
  __shared__ i32x4 red[3][MT][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = lane & 15, g = lane >> 4;
  const int n = blockIdx.x * 16 + c;
  const int nr = n < N ? n : N - 1;  // edge rows load a real row, never store
  const int nk = K >> 6;
  const int s0 = (w * nk) >> 2, s1 = ((w + 1) * nk) >> 2;
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
  for (int v = 0; v < 3; ++v)  // wave order: exact int32 sums
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
  if ((reinterpret_cast<uintptr_t>(W) & 15) || (reinterpret_cast<uintptr_t>(ws) & 15)) return hipErrorInvalidValue;
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
  if (Mp == 16)
    hipLaunchKernelGGL(i8_decode_gemv_kernel<1>, grid, dim3(kGemv), 0, s, xq, sx, W, sw, oidx, ocnt, xo, bias,
                       bias_dtype, y, y_dtype, M, N, K);
  else
    hipLaunchKernelGGL(i8_decode_gemv_kernel<2>, grid, dim3(kGemv), 0, s, xq, sx, W, sw, oidx, ocnt, xo, bias,
                       bias_dtype, y, y_dtype, M, N, K);
  return hipGetLastError();
}

}  // namespace ptdt
