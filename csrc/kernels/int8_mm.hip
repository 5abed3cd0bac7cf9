// LLM.int8 matrix multiply for gfx950: vector-wise int8 quantisation with the
// outlier decomposition of bitsandbytes (reference: BitsAndBytesConfig(load_in_8bit=True),
// NB03:52-56).
//
//   y = (Xq . Wq^T) * sx[m] * sw[n]  +  X[:, O] . Wdq[:, O]^T  (+ bias)
//
// O = the input features with |x| > threshold somewhere in the batch (column absmax);
// those columns are zeroed before the activation rows are quantised (absmax per row)
// and multiplied in 16/32-bit instead (the caller gathers them: usually a handful).
//   int8_col_outliers : column absmax > threshold -> mask[K]
//   int8_quant_rows   : per-row absmax over the non-outlier columns, q = rint(x / s)
//   int8_mm           : int32 products on v_mfma_i32_16x16x64_i8 (2x the bf16 rate, exact),
//                       dequantised in the fp32 epilogue with the addend (outlier part) and bias
// The MFMA's A and B fragments are read straight from global memory (16 contiguous
// bytes of a row per lane, the same k set for A and B in every lane group), so the
// kernel needs K % 16 == 0 and 16-byte aligned rows.
#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

using i32x4 = __attribute__((ext_vector_type(4))) int;
constexpr int kThreads = 256;

template <typename T>
__global__ void __launch_bounds__(kThreads) col_outlier_kernel(const T* __restrict__ x, int M, int K, float thr,
                                                               uint8_t* __restrict__ mask) {
  const int k = blockIdx.x * kThreads + threadIdx.x;
  if (k >= K) return;
  float amax = 0.f;
  for (int m = 0; m < M; ++m) amax = fmaxf(amax, fabsf(Cvt<T>::load(x, (int64_t)m * K + k)));
  mask[k] = amax > thr ? 1 : 0;
}

template <typename T>
__global__ void __launch_bounds__(kThreads) row_quant_kernel(const T* __restrict__ x, int K,
                                                             const uint8_t* __restrict__ mask, int8_t* __restrict__ q,
                                                             float* __restrict__ scale) {
  __shared__ float red[16];
  const int64_t r = blockIdx.x;
  const T* xr = x + r * K;
  float amax = 0.f;
  for (int k = threadIdx.x; k < K; k += kThreads)
    if (!(mask && mask[k])) amax = fmaxf(amax, fabsf(Cvt<T>::load(xr, k)));
  amax = block_max(amax, red);
  const float sc = amax > 0.f ? amax / 127.f : 1.f;
  const float inv = 1.f / sc;
  for (int k = threadIdx.x; k < K; k += kThreads) {
    float v = (mask && mask[k]) ? 0.f : rintf(Cvt<T>::load(xr, k) * inv);
    v = fminf(fmaxf(v, -127.f), 127.f);
    q[r * K + k] = (int8_t)v;
  }
  if (threadIdx.x == 0) scale[r] = sc;
}

// 64x64 output tile per workgroup, 4 waves of 32x32 (2x2 MFMA tiles of 16x16), K in steps of 64
__global__ void __launch_bounds__(kThreads) i8_mm_kernel(const int8_t* __restrict__ A, const float* __restrict__ sa,
                                                         const int8_t* __restrict__ B, const float* __restrict__ sb,
                                                         const float* __restrict__ addend, const void* bias,
                                                         int bias_bf16, int M, int N, int K, void* y, int y_bf16,
                                                         int tm, int tn) {
  const int tile = xcd_remap(blockIdx.x, tm * tn);
  const int m0 = (tile / tn) * 64, n0 = (tile % tn) * 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int c = lane & 15, g = lane >> 4;
  i32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = i32x4{0, 0, 0, 0};
  int ra[2], rb[2];
  bool va[2], vb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    ra[i] = m0 + wr * 32 + 16 * i + c;
    va[i] = ra[i] < M;
    rb[i] = n0 + wc * 32 + 16 * i + c;
    vb[i] = rb[i] < N;
  }
  for (int k0 = 0; k0 < K; k0 += 64) {
    const int k = k0 + 16 * g;  // this lane group's 16 consecutive k (same set for A and B)
    const bool kin = k < K;
    i32x4 a[2], b[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      a[i] = (va[i] && kin) ? *reinterpret_cast<const i32x4*>(A + (int64_t)ra[i] * K + k) : i32x4{0, 0, 0, 0};
      b[i] = (vb[i] && kin) ? *reinterpret_cast<const i32x4*>(B + (int64_t)rb[i] * K + k) : i32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  // D layout: [m = 4 g + r][n = c] of each 16x16 tile
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * 32 + 16 * i + 4 * g + r;
        const int n = n0 + wc * 32 + 16 * j + c;
        if (m < M && n < N) {
          float v = (float)acc[i][j][r] * sa[m] * sb[n];
          if (addend) v += addend[(int64_t)m * N + n];
          if (bias) v += bias_bf16 ? bf16_to_f32(static_cast<const uint16_t*>(bias)[n]) : static_cast<const float*>(bias)[n];
          if (y_bf16)
            static_cast<uint16_t*>(y)[(int64_t)m * N + n] = f32_to_bf16(v);
          else
            static_cast<float*>(y)[(int64_t)m * N + n] = v;
        }
      }
}

}  // namespace

hipError_t int8_col_outliers(const void* x, int dtype, int M, int K, float threshold, uint8_t* mask, hipStream_t s) {
  if (K <= 0) return hipSuccess;
  const dim3 grid((K + kThreads - 1) / kThreads);
  if (dtype == kF32)
    hipLaunchKernelGGL(col_outlier_kernel<float>, grid, dim3(kThreads), 0, s, (const float*)x, M, K, threshold, mask);
  else
    hipLaunchKernelGGL(col_outlier_kernel<uint16_t>, grid, dim3(kThreads), 0, s, (const uint16_t*)x, M, K, threshold,
                       mask);
  return hipGetLastError();
}

hipError_t int8_quant_rows(const void* x, int dtype, int M, int K, const uint8_t* mask, int8_t* q, float* scale,
                           hipStream_t s) {
  if (M <= 0 || K <= 0) return hipSuccess;
  if (dtype == kF32)
    hipLaunchKernelGGL(row_quant_kernel<float>, dim3(M), dim3(kThreads), 0, s, (const float*)x, K, mask, q, scale);
  else
    hipLaunchKernelGGL(row_quant_kernel<uint16_t>, dim3(M), dim3(kThreads), 0, s, (const uint16_t*)x, K, mask, q,
                       scale);
  return hipGetLastError();
}

hipError_t int8_mm(const int8_t* A, const float* sa, const int8_t* B, const float* sb, const float* addend,
                   const void* bias, int bias_bf16, int M, int N, int K, void* y, int y_dtype, hipStream_t s) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (K % 16 != 0) return hipErrorInvalidValue;
  const int tm = (M + 63) / 64, tn = (N + 63) / 64;
  hipLaunchKernelGGL(i8_mm_kernel, dim3(tm * tn), dim3(kThreads), 0, s, A, sa, B, sb, addend, bias, bias_bf16, M, N, K,
                     y, y_dtype == kBF16 ? 1 : 0, tm, tn);
  return hipGetLastError();
}

}  // namespace ptdt
