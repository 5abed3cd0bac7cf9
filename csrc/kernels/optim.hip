// Fused optimizer and DDP-bucket kernels (gfx950).
//
// Reference call sites: SGD ddp_gpus.py:39,82 / NB03:534,542,977,992 (foreach
// SGD over 2..161 tensors) and Adam NB01:287,487 (foreach Adam), DDP bucket
// copy+scale in the Reducer hooks.
//
// Two forms:
//  * *_flat: the framework keeps parameters / gradients / optimizer state in
//    contiguous flat buffers (FlatParameters), so one grid-stride launch with
//    16-byte vector accesses updates the whole model.
//  * *_multi: a kernel-argument tensor list (<= 32 tensors per launch, no
//    device-side metadata, so it is hipGraph-capturable); blocks are mapped
//    to (tensor, chunk) by a prefix search over chunk counts.
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

constexpr int kBlock = 256;
constexpr int kChunk = 4096;  // elements per block in multi-tensor launches

struct SgdHyper {
  float lr, mu, damp, wd, gscale;
  int nesterov;
};
struct AdamHyper {
  float lr, b1, b2, eps, wd, gscale;
  int decoupled;
};

__device__ __forceinline__ float sgd_update(float p, float g, float* mom, int64_t i, bool first,
                                            const SgdHyper& h) {
  g *= h.gscale;
  float d = g + h.wd * p;
  if (mom != nullptr && h.mu != 0.f) {
    const float buf = first ? d : h.mu * mom[i] + (1.f - h.damp) * d;
    mom[i] = buf;
    d = h.nesterov ? d + h.mu * buf : buf;
  }
  return p - h.lr * d;
}

// torch.optim.Adam(W) math, fp32 state.
__device__ __forceinline__ float adam_update(float p, float g, float* m, float* v, int64_t i,
                                             float bc1, float bc2_sqrt, const AdamHyper& h) {
  g *= h.gscale;
  if (h.decoupled) {
    p *= (1.f - h.lr * h.wd);
  } else {
    g += h.wd * p;
  }
  const float mi = h.b1 * m[i] + (1.f - h.b1) * g;
  const float vi = h.b2 * v[i] + (1.f - h.b2) * g * g;
  m[i] = mi;
  v[i] = vi;
  const float denom = sqrtf(vi) / bc2_sqrt + h.eps;
  return p - (h.lr / bc1) * (mi / denom);
}

__global__ void __launch_bounds__(kBlock) sgd_flat_kernel(float* __restrict__ p,
                                                          const float* __restrict__ g, float* mom,
                                                          int32_t* step, int64_t n, SgdHyper h) {
  const bool first = step ? (*step == 0) : false;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t t0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  // 4-wide vector body when aligned
  const int64_t n4 = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g)) & 15) == 0 &&
                             (mom == nullptr || (reinterpret_cast<uintptr_t>(mom) & 15) == 0)
                         ? n / 4
                         : 0;
  for (int64_t q = t0; q < n4; q += stride) {
    float4 pv = reinterpret_cast<float4*>(p)[q];
    const float4 gv = reinterpret_cast<const float4*>(g)[q];
    pv.x = sgd_update(pv.x, gv.x, mom, 4 * q + 0, first, h);
    pv.y = sgd_update(pv.y, gv.y, mom, 4 * q + 1, first, h);
    pv.z = sgd_update(pv.z, gv.z, mom, 4 * q + 2, first, h);
    pv.w = sgd_update(pv.w, gv.w, mom, 4 * q + 3, first, h);
    reinterpret_cast<float4*>(p)[q] = pv;
  }
  for (int64_t i = 4 * n4 + t0; i < n; i += stride) p[i] = sgd_update(p[i], g[i], mom, i, first, h);
}

__global__ void sgd_step_inc(int32_t* step) { *step += 1; }

__global__ void __launch_bounds__(kBlock) adam_flat_kernel(float* __restrict__ p,
                                                           const float* __restrict__ g, float* m,
                                                           float* v, const int32_t* step, int64_t n,
                                                           AdamHyper h) {
  const float t = (float)(*step);
  const float bc1 = 1.f - powf(h.b1, t);
  const float bc2s = sqrtf(1.f - powf(h.b2, t));
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    p[i] = adam_update(p[i], g[i], m, v, i, bc1, bc2s, h);
}

// ---------------------------------------------------------------- multi-tensor
__device__ __forceinline__ void locate_chunk(const int64_t* numel, int n, int blk, int& t,
                                             int64_t& start) {
  int acc = 0;
  for (t = 0; t < n; ++t) {
    const int c = (int)((numel[t] + kChunk - 1) / kChunk);
    if (blk < acc + c) break;
    acc += c;
  }
  start = (int64_t)(blk - acc) * kChunk;
}

template <typename T>
__global__ void __launch_bounds__(kBlock) sgd_multi_kernel(TensorList tl, int32_t* step,
                                                           SgdHyper h) {
  int t;
  int64_t start;
  locate_chunk(tl.numel, tl.n, blockIdx.x, t, start);
  if (t >= tl.n) return;
  const bool first = step ? (*step == 0) : false;
  T* p = static_cast<T*>(tl.p[t]);
  const T* g = static_cast<const T*>(tl.g[t]);
  float* mom = tl.s1[t];
  // f32 params: the bf16 autocast copy of the updated weight, written in the same pass
  uint16_t* shadow = std::is_same<T, float>::value ? reinterpret_cast<uint16_t*>(tl.s2[t]) : nullptr;
  const int64_t end = min(start + (int64_t)kChunk, tl.numel[t]);
  if constexpr (std::is_same<T, float>::value) {
    // 4 elements per thread: 16-B loads/stores of p, g, momentum and one 8-B store of the bf16 shadow,
    // when this tensor's pointers allow it (chunk starts are multiples of kChunk: aligned with them)
    const uintptr_t al = reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) |
                         reinterpret_cast<uintptr_t>(mom) | (reinterpret_cast<uintptr_t>(shadow) << 1);
    if ((al & 15) == 0 && (mom != nullptr || h.mu == 0.f)) {
      const int64_t vend = start + ((end - start) & ~(int64_t)3);
      for (int64_t i = start + 4 * threadIdx.x; i < vend; i += 4 * kBlock) {
        const float4 pv = *reinterpret_cast<const float4*>(p + i);
        const float4 gv = *reinterpret_cast<const float4*>(g + i);
        float pa[4] = {pv.x, pv.y, pv.z, pv.w};
        const float ga[4] = {gv.x, gv.y, gv.z, gv.w};
        float ma[4] = {0.f, 0.f, 0.f, 0.f};
        if (mom != nullptr && h.mu != 0.f && !first) {
          const float4 mv = *reinterpret_cast<const float4*>(mom + i);
          ma[0] = mv.x, ma[1] = mv.y, ma[2] = mv.z, ma[3] = mv.w;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float d = ga[k] * h.gscale + h.wd * pa[k];
          if (mom != nullptr && h.mu != 0.f) {
            ma[k] = first ? d : h.mu * ma[k] + (1.f - h.damp) * d;
            d = h.nesterov ? d + h.mu * ma[k] : ma[k];
          }
          pa[k] = pa[k] - h.lr * d;
        }
        *reinterpret_cast<float4*>(p + i) = make_float4(pa[0], pa[1], pa[2], pa[3]);
        if (mom != nullptr && h.mu != 0.f) *reinterpret_cast<float4*>(mom + i) = make_float4(ma[0], ma[1], ma[2], ma[3]);
        if (shadow) *reinterpret_cast<uint2*>(shadow + i) = make_uint2(pack_bf16x2(pa[0], pa[1]), pack_bf16x2(pa[2], pa[3]));
      }
      for (int64_t i = vend + threadIdx.x; i < end; i += kBlock) {  // tail (< 4 elements)
        const float nv = sgd_update(p[i], g[i], mom, i, first, h);
        p[i] = nv;
        if (shadow) shadow[i] = f32_to_bf16(nv);
      }
      return;
    }
  }
  for (int64_t i = start + threadIdx.x; i < end; i += kBlock) {
    const float pv = Cvt<T>::load(p, i);
    const float nv = sgd_update(pv, Cvt<T>::load(g, i), mom, i, first, h);
    Cvt<T>::store(p, i, nv);
    if (shadow) shadow[i] = f32_to_bf16(nv);
  }
}

template <typename T>
__global__ void __launch_bounds__(kBlock) adam_multi_kernel(TensorList tl, const int32_t* step,
                                                            AdamHyper h) {
  int t;
  int64_t start;
  locate_chunk(tl.numel, tl.n, blockIdx.x, t, start);
  if (t >= tl.n) return;
  const float st = (float)(*step);
  const float bc1 = 1.f - powf(h.b1, st);
  const float bc2s = sqrtf(1.f - powf(h.b2, st));
  T* p = static_cast<T*>(tl.p[t]);
  const T* g = static_cast<const T*>(tl.g[t]);
  const int64_t end = min(start + (int64_t)kChunk, tl.numel[t]);
  for (int64_t i = start + threadIdx.x; i < end; i += kBlock) {
    const float pv = Cvt<T>::load(p, i);
    Cvt<T>::store(p, i, adam_update(pv, Cvt<T>::load(g, i), tl.s1[t], tl.s2[t], i, bc1, bc2s, h));
  }
}

template <typename T>
__global__ void __launch_bounds__(kBlock) pack_kernel(CopyList cl, T* flat, float scale, int unpack) {
  int t;
  int64_t start;
  locate_chunk(cl.numel, cl.n, blockIdx.x, t, start);
  if (t >= cl.n) return;
  T* x = static_cast<T*>(cl.t[t]);
  const int64_t off = cl.offset[t];
  const int64_t end = min(start + (int64_t)kChunk, cl.numel[t]);
  for (int64_t i = start + threadIdx.x; i < end; i += kBlock) {
    if (unpack)
      Cvt<T>::store(x, i, Cvt<T>::load(flat, off + i) * scale);
    else
      Cvt<T>::store(flat, off + i, Cvt<T>::load(x, i) * scale);
  }
}

// dst[t][i] = f32(src[t][i]): bf16 weight gradients (autocast convolutions) into their f32 DDP bucket
// slots, one launch per bucket instead of one copy per parameter (ops/conv.py deferred casts)
__global__ void __launch_bounds__(kBlock) cast_bf16_f32_multi_kernel(TensorList tl) {
  int t;
  int64_t start;
  locate_chunk(tl.numel, tl.n, blockIdx.x, t, start);
  if (t >= tl.n) return;
  float* __restrict__ d = static_cast<float*>(tl.p[t]);
  const uint16_t* __restrict__ src = static_cast<const uint16_t*>(tl.g[t]);
  const int64_t end = min(start + (int64_t)kChunk, tl.numel[t]);
  for (int64_t i = start + threadIdx.x; i < end; i += kBlock) d[i] = bf16_to_f32(src[i]);
}

template <typename T>
__global__ void __launch_bounds__(kBlock) scale_kernel(T* x, int64_t n, float scale) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    Cvt<T>::store(x, i, Cvt<T>::load(x, i) * scale);
}

inline int grid_for(int64_t n, int per_thread = 4) {
  int64_t g = (n + (int64_t)kBlock * per_thread - 1) / ((int64_t)kBlock * per_thread);
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;  // 256 CUs x 8 blocks, grid-stride the rest
  return (int)g;
}
template <typename L>
int chunk_blocks(const L& l) {
  int b = 0;
  for (int i = 0; i < l.n; ++i) b += (int)((l.numel[i] + kChunk - 1) / kChunk);
  return b;
}

}  // namespace

hipError_t sgd_flat(float* p, const float* g, float* mom, int32_t* step, int64_t n, float lr,
                    float momentum, float dampening, float weight_decay, int nesterov,
                    float grad_scale, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  SgdHyper h{lr, momentum, dampening, weight_decay, grad_scale, nesterov};
  hipLaunchKernelGGL(sgd_flat_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, p, g, mom, step, n, h);
  if (step) hipLaunchKernelGGL(sgd_step_inc, dim3(1), dim3(1), 0, s, step);
  return hipGetLastError();
}

hipError_t adam_flat(float* p, const float* g, float* m, float* v, const int32_t* step, int64_t n,
                     float lr, float beta1, float beta2, float eps, float weight_decay,
                     int decoupled, float grad_scale, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  AdamHyper h{lr, beta1, beta2, eps, weight_decay, grad_scale, decoupled};
  hipLaunchKernelGGL(adam_flat_kernel, dim3(grid_for(n, 1)), dim3(kBlock), 0, s, p, g, m, v, step, n, h);
  return hipGetLastError();
}

hipError_t sgd_multi(const TensorList& tl, int dtype, int32_t* step, float lr, float momentum,
                     float dampening, float weight_decay, int nesterov, float grad_scale,
                     hipStream_t s) {
  const int nb = chunk_blocks(tl);
  if (nb == 0) return hipSuccess;
  SgdHyper h{lr, momentum, dampening, weight_decay, grad_scale, nesterov};
  if (dtype == kF32)
    hipLaunchKernelGGL(sgd_multi_kernel<float>, dim3(nb), dim3(kBlock), 0, s, tl, step, h);
  else
    hipLaunchKernelGGL(sgd_multi_kernel<uint16_t>, dim3(nb), dim3(kBlock), 0, s, tl, step, h);
  return hipGetLastError();
}

hipError_t adam_multi(const TensorList& tl, int dtype, const int32_t* step, float lr, float beta1,
                      float beta2, float eps, float weight_decay, int decoupled, float grad_scale,
                      hipStream_t s) {
  const int nb = chunk_blocks(tl);
  if (nb == 0) return hipSuccess;
  AdamHyper h{lr, beta1, beta2, eps, weight_decay, grad_scale, decoupled};
  if (dtype == kF32)
    hipLaunchKernelGGL(adam_multi_kernel<float>, dim3(nb), dim3(kBlock), 0, s, tl, step, h);
  else
    hipLaunchKernelGGL(adam_multi_kernel<uint16_t>, dim3(nb), dim3(kBlock), 0, s, tl, step, h);
  return hipGetLastError();
}

hipError_t bucket_pack(const CopyList& cl, void* flat, int dtype, float scale, hipStream_t s) {
  const int nb = chunk_blocks(cl);
  if (nb == 0) return hipSuccess;
  if (dtype == kF32)
    hipLaunchKernelGGL(pack_kernel<float>, dim3(nb), dim3(kBlock), 0, s, cl, (float*)flat, scale, 0);
  else
    hipLaunchKernelGGL(pack_kernel<uint16_t>, dim3(nb), dim3(kBlock), 0, s, cl, (uint16_t*)flat, scale, 0);
  return hipGetLastError();
}

hipError_t bucket_unpack(const CopyList& cl, const void* flat, int dtype, float scale, hipStream_t s) {
  const int nb = chunk_blocks(cl);
  if (nb == 0) return hipSuccess;
  if (dtype == kF32)
    hipLaunchKernelGGL(pack_kernel<float>, dim3(nb), dim3(kBlock), 0, s, cl, (float*)flat, scale, 1);
  else
    hipLaunchKernelGGL(pack_kernel<uint16_t>, dim3(nb), dim3(kBlock), 0, s, cl, (uint16_t*)flat, scale, 1);
  return hipGetLastError();
}

hipError_t cast_bf16_f32_multi(const TensorList& tl, hipStream_t s) {
  const int nb = chunk_blocks(tl);
  if (nb == 0) return hipSuccess;
  hipLaunchKernelGGL(cast_bf16_f32_multi_kernel, dim3(nb), dim3(kBlock), 0, s, tl);
  return hipGetLastError();
}

hipError_t scale_inplace(void* x, int64_t n, int dtype, float scale, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (dtype == kF32)
    hipLaunchKernelGGL(scale_kernel<float>, dim3(grid_for(n)), dim3(kBlock), 0, s, (float*)x, n, scale);
  else
    hipLaunchKernelGGL(scale_kernel<uint16_t>, dim3(grid_for(n)), dim3(kBlock), 0, s, (uint16_t*)x, n, scale);
  return hipGetLastError();
}

}  // namespace ptdt
