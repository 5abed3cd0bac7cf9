// Max pooling over NHWC (channels_last) activations: forward with a one-byte
// window argmax, backward as a deterministic gather (no atomics, no int64
// index tensor).
//
// Why: ResNet-50's stem pool (3x3 / stride 2 / pad 1 over [B, 112, 112, 64])
// took ~0.45 ms of the bf16 B=128 DDP step in PyTorch-ROCm's NHWC kernels
// (profiles/r1_resnet_window.md), whose backward scatters through 8-byte
// indices. Here each thread owns 16 B of channels (8 bf16 / 4 f32) of one
// output pixel (forward) or one input pixel (backward): the forward reads the
// window with 16-B loads and writes y plus an argmax byte per element
// (window offset dy*kw + dx); the backward visits the <= ceil(k/s)^2 output
// windows covering its pixel and adds the dy entries whose argmax points at it.
// NaN propagates like torch (a NaN wins the max).
#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

constexpr int kThreads = 256;

template <typename T>
struct V16 {
  static constexpr int V = 16 / sizeof(T);
  __device__ __forceinline__ static void load(const T* p, float (&v)[V]) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
    if constexpr (sizeof(T) == 4) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = __uint_as_float(w[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
      }
    }
  }
  __device__ __forceinline__ static void store(T* p, const float (&v)[V]) {
    uint32_t w[4];
    if constexpr (sizeof(T) == 4) {
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = __float_as_uint(v[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f32_to_bf16(v[2 * i]) | ((uint32_t)f32_to_bf16(v[2 * i + 1]) << 16);
    }
    *reinterpret_cast<uint4*>(p) = uint4{w[0], w[1], w[2], w[3]};
  }
};

// AFF: the BatchNorm apply (+ReLU) of the pool's input done on load (PoolArgs.scale/shift/relu), with
// the same fmaf and rounding as batchnorm.hip's apply pass: output and argmax are bit-identical to
// BN-then-pool, without writing and re-reading the normalised activation.
template <typename T>
__device__ __forceinline__ float round_to(float v) {
  if constexpr (sizeof(T) == 4) return v;
  else return __uint_as_float((uint32_t)f32_to_bf16(v) << 16);
}

template <typename T, bool AFF>
__global__ void __launch_bounds__(kThreads) maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                               uint8_t* __restrict__ arg, PoolArgs a) {
  constexpr int V = V16<T>::V;
  const int cv = a.C / V;
  const int64_t total = (int64_t)a.N * a.Ho * a.Wo * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int c0 = (int)(t % cv) * V;
    int64_t pix = t / cv;
    const int wo = (int)(pix % a.Wo);
    pix /= a.Wo;
    const int ho = (int)(pix % a.Ho);
    const int n = (int)(pix / a.Ho);
    float best[V];
    uint32_t bi[V];
    float sc[AFF ? V : 1], sf[AFF ? V : 1];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      best[v] = -__builtin_inff();
      bi[v] = 0;
      if constexpr (AFF) {
        sc[v] = a.scale[c0 + v];
        sf[v] = a.shift[c0 + v];
      }
    }
    const int h0 = ho * a.sh - a.ph, w0 = wo * a.sw - a.pw;
    for (int dy = 0; dy < a.kh; ++dy) {
      const int h = h0 + dy;
      if (h < 0 || h >= a.H) continue;
      for (int dx = 0; dx < a.kw; ++dx) {
        const int w = w0 + dx;
        if (w < 0 || w >= a.W) continue;
        float v_[V];
        V16<T>::load(x + (((int64_t)n * a.H + h) * a.W + w) * a.C + c0, v_);
        if constexpr (AFF) {
#pragma unroll
          for (int v = 0; v < V; ++v) {
            float o = fmaf(v_[v], sc[v], sf[v]);
            if (a.relu) o = fmaxf(o, 0.f);
            v_[v] = round_to<T>(o);
          }
        }
        const uint32_t k = (uint32_t)(dy * a.kw + dx);
#pragma unroll
        for (int v = 0; v < V; ++v)
          if (v_[v] > best[v] || v_[v] != v_[v]) {  // NaN wins (and stays: NaN > x is false)
            if (best[v] == best[v]) {
              best[v] = v_[v];
              bi[v] = k;
            }
          }
      }
    }
    const int64_t o = (((int64_t)n * a.Ho + ho) * a.Wo + wo) * a.C + c0;
    V16<T>::store(y + o, best);
    if constexpr (V == 8) {
      uint2 packed;
      packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
      packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
      *reinterpret_cast<uint2*>(arg + o) = packed;
    } else {
      *reinterpret_cast<uint32_t*>(arg + o) = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(kThreads) maxpool_bwd_kernel(const T* __restrict__ gy,
                                                               const uint8_t* __restrict__ arg, T* __restrict__ gx,
                                                               PoolArgs a) {
  constexpr int V = V16<T>::V;
  const int cv = a.C / V;
  const int64_t total = (int64_t)a.N * a.H * a.W * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int c0 = (int)(t % cv) * V;
    int64_t pix = t / cv;
    const int w = (int)(pix % a.W);
    pix /= a.W;
    const int h = (int)(pix % a.H);
    const int n = (int)(pix / a.H);
    // output windows covering (h, w): ho*sh - ph <= h <= ho*sh - ph + kh - 1
    const int hp = h + a.ph, wp = w + a.pw;
    const int ho_lo = hp - a.kh + 1 > 0 ? (hp - a.kh + 1 + a.sh - 1) / a.sh : 0;
    const int ho_hi = min(hp / a.sh, a.Ho - 1);
    const int wo_lo = wp - a.kw + 1 > 0 ? (wp - a.kw + 1 + a.sw - 1) / a.sw : 0;
    const int wo_hi = min(wp / a.sw, a.Wo - 1);
    float acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = 0.f;
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        const uint32_t k = (uint32_t)((hp - ho * a.sh) * a.kw + (wp - wo * a.sw));
        const int64_t o = (((int64_t)n * a.Ho + ho) * a.Wo + wo) * a.C + c0;
        uint32_t b[2];
        if constexpr (V == 8) {
          const uint2 p = *reinterpret_cast<const uint2*>(arg + o);
          b[0] = p.x;
          b[1] = p.y;
        } else {
          b[0] = *reinterpret_cast<const uint32_t*>(arg + o);
          b[1] = 0;
        }
        float g[V];
        V16<T>::load(gy + o, g);
#pragma unroll
        for (int v = 0; v < V; ++v)
          if (((b[v >> 2] >> (8 * (v & 3))) & 0xffu) == k) acc[v] += g[v];
      }
    }
    V16<T>::store(gx + (((int64_t)n * a.H + h) * a.W + w) * a.C + c0, acc);
  }
}

int grid_for(int64_t work) {
  int64_t b = (work + kThreads * 2 - 1) / (kThreads * 2);
  if (b > 8192) b = 8192;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace

hipError_t maxpool2d_nhwc_forward(const void* x, void* y, uint8_t* argmax, int dtype, const PoolArgs& a,
                                  hipStream_t s) {
  const int V = dtype == kF32 ? 4 : 8;
  if (a.C % V || a.kh * a.kw > 256 || a.kh < 1 || a.kw < 1 || a.sh < 1 || a.sw < 1) return hipErrorInvalidValue;
  const int64_t work = (int64_t)a.N * a.Ho * a.Wo * (a.C / V);
  if (work == 0) return hipSuccess;
  if ((a.scale == nullptr) != (a.shift == nullptr)) return hipErrorInvalidValue;
  const bool aff = a.scale != nullptr;
  if (dtype == kF32) {
    if (aff)
      hipLaunchKernelGGL((maxpool_fwd_kernel<float, true>), dim3(grid_for(work)), dim3(kThreads), 0, s,
                         static_cast<const float*>(x), static_cast<float*>(y), argmax, a);
    else
      hipLaunchKernelGGL((maxpool_fwd_kernel<float, false>), dim3(grid_for(work)), dim3(kThreads), 0, s,
                         static_cast<const float*>(x), static_cast<float*>(y), argmax, a);
  } else {
    if (aff)
      hipLaunchKernelGGL((maxpool_fwd_kernel<uint16_t, true>), dim3(grid_for(work)), dim3(kThreads), 0, s,
                         static_cast<const uint16_t*>(x), static_cast<uint16_t*>(y), argmax, a);
    else
      hipLaunchKernelGGL((maxpool_fwd_kernel<uint16_t, false>), dim3(grid_for(work)), dim3(kThreads), 0, s,
                         static_cast<const uint16_t*>(x), static_cast<uint16_t*>(y), argmax, a);
  }
  return hipGetLastError();
}

hipError_t maxpool2d_nhwc_backward(const void* gy, const uint8_t* argmax, void* gx, int dtype, const PoolArgs& a,
                                   hipStream_t s) {
  const int V = dtype == kF32 ? 4 : 8;
  if (a.C % V || a.kh * a.kw > 256 || a.sh < 1 || a.sw < 1) return hipErrorInvalidValue;
  const int64_t work = (int64_t)a.N * a.H * a.W * (a.C / V);
  if (work == 0) return hipSuccess;
  if (dtype == kF32)
    hipLaunchKernelGGL(maxpool_bwd_kernel<float>, dim3(grid_for(work)), dim3(kThreads), 0, s,
                       static_cast<const float*>(gy), argmax, static_cast<float*>(gx), a);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<uint16_t>, dim3(grid_for(work)), dim3(kThreads), 0, s,
                       static_cast<const uint16_t*>(gy), argmax, static_cast<uint16_t*>(gx), a);
  return hipGetLastError();
}

}  // namespace ptdt
