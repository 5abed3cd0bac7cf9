// Int8 weight-only quantisation and GEMM (gfx950).
//
// Reference: LlamaForCausalLM.from_pretrained(..., BitsAndBytesConfig(load_in_8bit=True),
// device_map="auto") NB03:52-56. bitsandbytes quantises each
// projection weight row-wise (absmax) when it moves to the GPU. Here:
//   quantize_rowwise_int8: one workgroup per output row, wave64 absmax, q = rint(w*127/absmax).
//   int8_weight_gemm     : y[M,N] = x[M,K] . (q[N,K] * s[N])^T (+ bias).
// Integers in [-127, 127] are exact in bf16, so the int8 tile is widened to
// bf16 while staging into LDS and multiplied on v_mfma_f32_16x16x32_bf16; the
// per-row scale is applied once in the fp32 epilogue (no dequantised weight
// copy ever exists in HBM: 1 byte/weight is read, half of bf16).
#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
constexpr int kThreads = 256;

template <typename T>
__global__ void __launch_bounds__(kThreads) quant_kernel(const T* w, int64_t cols, int8_t* q, float* scale) {
  __shared__ float red[16];
  const int64_t r = blockIdx.x;
  const T* wr = w + r * cols;
  float amax = 0.f;
  for (int64_t c = threadIdx.x; c < cols; c += kThreads) amax = fmaxf(amax, fabsf(Cvt<T>::load(wr, c)));
  amax = block_max(amax, red);
  const float sc = amax > 0.f ? amax / 127.f : 1.f;
  for (int64_t c = threadIdx.x; c < cols; c += kThreads) {
    float v = rintf(Cvt<T>::load(wr, c) / sc);  // IEEE division: the reference's round(w / s) bit for bit
    v = fminf(fmaxf(v, -127.f), 127.f);
    q[r * cols + c] = (int8_t)v;
  }
  if (threadIdx.x == 0) scale[r] = sc;
}

template <typename TX>
__global__ void __launch_bounds__(kThreads) w8_gemm_kernel(const TX* x, const int8_t* q, const float* scale,
                                                           const void* bias, int bias_bf16, int M, int N,
                                                           int K, void* y, int y_bf16, int tm, int tn) {
  constexpr int BM = 64, BN = 64, BK = 32, LDK = BK + 8;
  __shared__ __attribute__((aligned(16))) uint16_t As[BM * LDK];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[BN * LDK];
  const int tile = xcd_remap(blockIdx.x, tm * tn);
  const int m0 = (tile / tn) * BM, n0 = (tile % tn) * BN;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < K; k0 += BK) {
#pragma unroll
    for (int j = 0; j < (BM * BK) / kThreads; ++j) {
      const int e = j * kThreads + threadIdx.x;
      const int r = e / BK, k = e % BK;
      const int gm = m0 + r, gk = k0 + k;
      As[r * LDK + k] = (gm < M && gk < K) ? f32_to_bf16(Cvt<TX>::load(x, (int64_t)gm * K + gk)) : 0;
      const int gn = n0 + r;
      Bs[r * LDK + k] = (gn < N && gk < K) ? f32_to_bf16((float)q[(int64_t)gn * K + gk]) : 0;
    }
    __syncthreads();
    bf16x8_t af[2], bfr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
      af[i] = *reinterpret_cast<const bf16x8_t*>(&As[(wr * 32 + i * 16 + (lane & 15)) * LDK + 8 * (lane >> 4)]);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      bfr[j] = *reinterpret_cast<const bf16x8_t*>(&Bs[(wc * 32 + j * 16 + (lane & 15)) * LDK + 8 * (lane >> 4)]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int n = n0 + wc * 32 + j * 16 + (lane & 15);
        if (m < M && n < N) {
          float v = acc[i][j][r] * scale[n];
          if (bias) v += bias_bf16 ? bf16_to_f32(static_cast<const uint16_t*>(bias)[n])
                                   : static_cast<const float*>(bias)[n];
          if (y_bf16)
            static_cast<uint16_t*>(y)[(int64_t)m * N + n] = f32_to_bf16(v);
          else
            static_cast<float*>(y)[(int64_t)m * N + n] = v;
        }
      }
}

}  // namespace

hipError_t quantize_rowwise_int8(const void* w, int dtype, int64_t rows, int64_t cols, int8_t* q,
                                 float* scale, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  if (dtype == kF32)
    hipLaunchKernelGGL(quant_kernel<float>, dim3((unsigned)rows), dim3(kThreads), 0, s, (const float*)w,
                       cols, q, scale);
  else
    hipLaunchKernelGGL(quant_kernel<uint16_t>, dim3((unsigned)rows), dim3(kThreads), 0, s,
                       (const uint16_t*)w, cols, q, scale);
  return hipGetLastError();
}

hipError_t int8_weight_gemm(const void* x, int x_dtype, const int8_t* q, const float* scale,
                            const void* bias, int M, int N, int K, void* y, int y_dtype,
                            hipStream_t s) {
  if (M <= 0 || N <= 0) return hipSuccess;
  const int tm = (M + 63) / 64, tn = (N + 63) / 64;
  // bias follows the activation dtype
  const int bias_bf16 = x_dtype == kBF16;
  if (x_dtype == kF32)
    hipLaunchKernelGGL(w8_gemm_kernel<float>, dim3(tm * tn), dim3(kThreads), 0, s, (const float*)x, q,
                       scale, bias, bias_bf16, M, N, K, y, y_dtype == kBF16, tm, tn);
  else
    hipLaunchKernelGGL(w8_gemm_kernel<uint16_t>, dim3(tm * tn), dim3(kThreads), 0, s,
                       (const uint16_t*)x, q, scale, bias, bias_bf16, M, N, K, y, y_dtype == kBF16, tm, tn);
  return hipGetLastError();
}

}  // namespace ptdt
