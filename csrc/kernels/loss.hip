// Loss kernels (gfx950): cross-entropy with soft or index targets, MSE.
//
// Reference call sites: F.cross_entropy ddp_gpus.py:37 ([B,1] logits with float
// targets -> soft-target CE), nn.MSELoss NB03:533,976 (K12/K16).
// One workgroup per row for CE (wave64 butterfly max/sum over the classes,
// inputs read once with vector loads into registers when C is small), and a
// grid-stride partial-sum + single-atomic reduction for MSE.
#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

constexpr int kBlock = 256;

template <typename T>
__global__ void __launch_bounds__(kBlock) ce_fwd_kernel(const T* __restrict__ logits,
                                                        const float* __restrict__ soft,
                                                        const int64_t* __restrict__ index, int B,
                                                        int C, int ignore_index, float ls,
                                                        float* __restrict__ row_loss,
                                                        float* __restrict__ lse_out) {
  __shared__ float red[16];
  const int b = blockIdx.x;
  const T* z = logits + (int64_t)b * C;
  float m = -INFINITY;
  for (int c = threadIdx.x; c < C; c += kBlock) m = fmaxf(m, Cvt<T>::load(z, c));
  m = block_max(m, red);
  float se = 0.f, zsum = 0.f, tz = 0.f, ts = 0.f;
  for (int c = threadIdx.x; c < C; c += kBlock) {
    const float zc = Cvt<T>::load(z, c);
    se += expf(zc - m);
    zsum += zc;
    if (soft) {
      const float t = soft[(int64_t)b * C + c];
      tz += t * zc;
      ts += t;
    }
  }
  se = block_sum(se, red);
  zsum = block_sum(zsum, red + 8);
  if (soft) {
    tz = block_sum(tz, red);
    ts = block_sum(ts, red + 8);
  }
  if (threadIdx.x == 0) {
    const float lse = m + logf(se);
    lse_out[b] = lse;
    lse_out[2 * B + b] = ts;  // row sum of soft targets, reused by the backward
    float l;
    if (soft) {
      // -sum_c t_c * (z_c - lse), label smoothing mixes in the uniform target
      l = -(tz - lse * ts);
      if (ls > 0.f) l = (1.f - ls) * l + ls * (lse - zsum / (float)C);
      row_loss[b] = l;
    } else {
      const int64_t y = index[b];
      if (y == ignore_index) {
        row_loss[b] = 0.f;
      } else {
        l = lse - Cvt<T>::load(z, y);
        if (ls > 0.f) l = (1.f - ls) * l + ls * (lse - zsum / (float)C);
        row_loss[b] = l;
      }
    }
  }
}

// Mean over rows (valid rows for index targets); single workgroup.
__global__ void __launch_bounds__(kBlock) ce_reduce_kernel(const float* row_loss,
                                                           const int64_t* index, int B,
                                                           int ignore_index, float* loss,
                                                           float* valid) {
  __shared__ float red[16];
  float s = 0.f, n = 0.f;
  for (int b = threadIdx.x; b < B; b += kBlock) {
    s += row_loss[b];
    n += (index == nullptr || index[b] != ignore_index) ? 1.f : 0.f;
  }
  s = block_sum(s, red);
  n = block_sum(n, red + 8);
  if (threadIdx.x == 0) {
    *loss = n > 0.f ? s / n : NAN;
    *valid = n;
  }
}

template <typename T>
__global__ void __launch_bounds__(kBlock) ce_bwd_kernel(const T* __restrict__ logits,
                                                        const float* __restrict__ soft,
                                                        const int64_t* __restrict__ index,
                                                        const float* __restrict__ lse,
                                                        const float* __restrict__ valid,
                                                        const float* __restrict__ grad_out, int B,
                                                        int C, int ignore_index, float ls,
                                                        T* __restrict__ dlogits) {
  const int64_t n = (int64_t)B * C;
  const float g = (grad_out ? *grad_out : 1.f) / fmaxf(*valid, 1.f);
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += stride) {
    const int b = (int)(e / C), c = (int)(e % C);
    const float p = expf(Cvt<T>::load(logits, e) - lse[b]);
    float d;
    if (soft) {
      // d/dz of -sum t (z - lse) = p * sum(t) - t (row sum saved by the forward)
      d = p * lse[2 * B + b] - soft[e];
      if (ls > 0.f) d = (1.f - ls) * d + ls * (p - 1.f / (float)C);
    } else {
      const int64_t y = index[b];
      if (y == ignore_index) {
        d = 0.f;
      } else {
        d = p - (c == y ? 1.f : 0.f);
        if (ls > 0.f) d = (1.f - ls) * d + ls * (p - 1.f / (float)C);
      }
    }
    Cvt<T>::store(dlogits, e, d * g);
  }
}

template <typename T>
__global__ void __launch_bounds__(kBlock) mse_fwd_kernel(const T* x, const T* y, int64_t n,
                                                         float* partial) {
  __shared__ float red[16];
  float s = 0.f;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const float d = Cvt<T>::load(x, i) - Cvt<T>::load(y, i);
    s = fmaf(d, d, s);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ void __launch_bounds__(kBlock) mse_finish_kernel(const float* partial, int np, int64_t n,
                                                            float* loss) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < np; i += kBlock) s += partial[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) *loss = s / (float)n;
}

template <typename T>
__global__ void __launch_bounds__(kBlock) mse_bwd_kernel(const T* x, const T* y, int64_t n,
                                                         const float* grad_out, T* dx, T* dy) {
  const float g = 2.f * (grad_out ? *grad_out : 1.f) / (float)n;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const float d = (Cvt<T>::load(x, i) - Cvt<T>::load(y, i)) * g;
    if (dx) Cvt<T>::store(dx, i, d);
    if (dy) Cvt<T>::store(dy, i, -d);
  }
}

inline int grid_for(int64_t n) {
  int64_t g = (n + kBlock * 4 - 1) / (kBlock * 4);
  return (int)(g < 1 ? 1 : (g > 1024 ? 1024 : g));
}

}  // namespace

// `lse` must hold 3*B floats: [logsumexp | per-row loss | soft-target row sums];
// `valid_count` and `loss` one float each.
hipError_t ce_forward(const void* logits, int dtype, const float* soft, const int64_t* index,
                      int B, int C, int ignore_index, float label_smoothing, float* loss,
                      float* lse, float* valid_count, hipStream_t s) {
  if (B <= 0 || C <= 0) return hipErrorInvalidValue;
  float* rows = lse + B;
  if (dtype == kF32)
    hipLaunchKernelGGL(ce_fwd_kernel<float>, dim3(B), dim3(kBlock), 0, s, (const float*)logits,
                       soft, index, B, C, ignore_index, label_smoothing, rows, lse);
  else
    hipLaunchKernelGGL(ce_fwd_kernel<uint16_t>, dim3(B), dim3(kBlock), 0, s,
                       (const uint16_t*)logits, soft, index, B, C, ignore_index, label_smoothing,
                       rows, lse);
  hipLaunchKernelGGL(ce_reduce_kernel, dim3(1), dim3(kBlock), 0, s, rows, soft ? nullptr : index, B,
                     ignore_index, loss, valid_count);
  return hipGetLastError();
}

hipError_t ce_backward(const void* logits, int dtype, const float* soft, const int64_t* index,
                       const float* lse, const float* valid_count, const float* grad_out, int B,
                       int C, int ignore_index, float label_smoothing, void* dlogits,
                       hipStream_t s) {
  const int64_t n = (int64_t)B * C;
  if (dtype == kF32)
    hipLaunchKernelGGL(ce_bwd_kernel<float>, dim3(grid_for(n)), dim3(kBlock), 0, s,
                       (const float*)logits, soft, index, lse, valid_count, grad_out, B, C,
                       ignore_index, label_smoothing, (float*)dlogits);
  else
    hipLaunchKernelGGL(ce_bwd_kernel<uint16_t>, dim3(grid_for(n)), dim3(kBlock), 0, s,
                       (const uint16_t*)logits, soft, index, lse, valid_count, grad_out, B, C,
                       ignore_index, label_smoothing, (uint16_t*)dlogits);
  return hipGetLastError();
}

// `loss` must point at 1 + 1024 floats (scalar + partial sums workspace).
hipError_t mse_forward(const void* x, const void* y, int dtype, int64_t n, float* loss,
                       hipStream_t s) {
  if (n <= 0) return hipErrorInvalidValue;
  const int g = grid_for(n);
  float* partial = loss + 1;
  if (dtype == kF32)
    hipLaunchKernelGGL(mse_fwd_kernel<float>, dim3(g), dim3(kBlock), 0, s, (const float*)x,
                       (const float*)y, n, partial);
  else
    hipLaunchKernelGGL(mse_fwd_kernel<uint16_t>, dim3(g), dim3(kBlock), 0, s, (const uint16_t*)x,
                       (const uint16_t*)y, n, partial);
  hipLaunchKernelGGL(mse_finish_kernel, dim3(1), dim3(kBlock), 0, s, partial, g, n, loss);
  return hipGetLastError();
}

hipError_t mse_backward(const void* x, const void* y, int dtype, int64_t n, const float* grad_out,
                        void* dx, void* dy, hipStream_t s) {
  if (dtype == kF32)
    hipLaunchKernelGGL(mse_bwd_kernel<float>, dim3(grid_for(n)), dim3(kBlock), 0, s,
                       (const float*)x, (const float*)y, n, grad_out, (float*)dx, (float*)dy);
  else
    hipLaunchKernelGGL(mse_bwd_kernel<uint16_t>, dim3(grid_for(n)), dim3(kBlock), 0, s,
                       (const uint16_t*)x, (const uint16_t*)y, n, grad_out, (uint16_t*)dx,
                       (uint16_t*)dy);
  return hipGetLastError();
}

}  // namespace ptdt
