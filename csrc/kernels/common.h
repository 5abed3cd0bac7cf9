// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels of this framework.
//
// Everything here assumes 64-lane wavefronts (CDNA), never 32-lane warps:
// cross-lane reductions use 6 butterfly steps, block sizes are multiples of 64.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define PTDT_WAVE 64

#define PTDT_HIP_CHECK(expr)                                                        \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess) return _e;                                                \
  } while (0)

namespace ptdt {

// ---------------------------------------------------------------- bf16 <-> f32
// bf16 is stored as raw uint16_t in every kernel signature (no vendor types in
// the ABI), converted with round-to-nearest-even.
__device__ __forceinline__ float bf16_to_f32(uint16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return 0x7fc0;  // NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

template <typename T> struct Cvt;
template <> struct Cvt<float> {
  __device__ __forceinline__ static float load(const float* p, int64_t i) { return p[i]; }
  __device__ __forceinline__ static void store(float* p, int64_t i, float v) { p[i] = v; }
};
template <> struct Cvt<uint16_t> {
  __device__ __forceinline__ static float load(const uint16_t* p, int64_t i) { return bf16_to_f32(p[i]); }
  __device__ __forceinline__ static void store(uint16_t* p, int64_t i, float v) { p[i] = f32_to_bf16(v); }
};

// ----------------------------------------------------------- wave64 reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, PTDT_WAVE);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, PTDT_WAVE));
  return v;
}

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024). `scratch` needs
// blockDim.x/64 floats of LDS. Result is valid in every thread.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  return r;
}
__device__ __forceinline__ float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, scratch[i]);
  return r;
}

// XCD-aware bijective remap of a 1-D workgroup id (cdna_hip_programming.md T1):
// consecutive logical tiles land on the same XCD (shared L2) instead of being
// round-robined over the 8 XCDs. Pure speed choice, never correctness.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  constexpr int NX = 8;
  if (nwg <= NX) return orig;
  const int q = nwg / NX, r = nwg % NX, xcd = orig % NX;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / NX;
}

}  // namespace ptdt
