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

// Explicit global address space for pointers that arrive inside by-value
// argument structs: the compiler cannot infer it there and would emit flat_*
// instructions (slower, and counted in lgkmcnt as well as vmcnt).
#define PTDT_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ const T PTDT_GLOBAL* gptr(const T* p) {
  return (const T PTDT_GLOBAL*)p;
}
template <typename T>
__device__ __forceinline__ T PTDT_GLOBAL* gptr_w(T* p) {
  return (T PTDT_GLOBAL*)p;
}

__host__ __device__ __forceinline__ int al4(int n) { return (n + 3) & ~3; }

// ---------------------------------------------------------------- bf16 <-> f32
// bf16 is stored as raw uint16_t in every kernel signature (no vendor types in
// the ABI), converted with round-to-nearest-even.
__device__ __forceinline__ float bf16_to_f32(uint16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}
// gfx950 converts in hardware: v_cvt_pk_bf16_f32 (round to nearest even, NaN stays NaN) -- one
// instruction instead of the 5-6 of a software rounding (profiles/r3_convbn.md)
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}
// two values -> one packed word (lo = a), one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) float f2_t;
  typedef __attribute__((ext_vector_type(2))) __bf16 bf2_t;
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2_t){a, b}, bf2_t));
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
// IEEE half (kF16): the LLM.int8 path's activations (the reference's load_in_8bit Llama runs in fp16)
template <> struct Cvt<_Float16> {
  __device__ __forceinline__ static float load(const _Float16* p, int64_t i) { return (float)p[i]; }
  __device__ __forceinline__ static void store(_Float16* p, int64_t i, float v) { p[i] = (_Float16)v; }
};

// ----------------------------------------------------------- wave64 reductions
// DPP / permlane based: every step is one VALU instruction (v_add_f32_dpp,
// v_permlane16/32_swap) instead of an LDS-crossbar ds_bpermute round trip
// (what __shfl_xor lowers to). All 64 lanes must be active.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141; // lane i <-> 7-i within 8 (pairs the two quads)
constexpr int kDppMirror = 0x140;     // lane i <-> 15-i within 16 (pairs the two halves)

// sum over aligned groups of G lanes (G in 1,2,4,8,16); result in every lane of the group
template <int G>
__device__ __forceinline__ float group_sum(float v) {
  if constexpr (G >= 2) v += dpp_f<kDppXor1>(v);
  if constexpr (G >= 4) v += dpp_f<kDppXor2>(v);
  if constexpr (G >= 8) v += dpp_f<kDppHalfMirror>(v);
  if constexpr (G >= 16) v += dpp_f<kDppMirror>(v);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
  v = group_sum<16>(v);
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  v = __int_as_float(p[0]) + __int_as_float(p[1]);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(q[0]) + __int_as_float(q[1]);
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_f<kDppXor1>(v));
  v = fmaxf(v, dpp_f<kDppXor2>(v));
  v = fmaxf(v, dpp_f<kDppHalfMirror>(v));
  v = fmaxf(v, dpp_f<kDppMirror>(v));
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  v = fmaxf(__int_as_float(p[0]), __int_as_float(p[1]));
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return fmaxf(__int_as_float(q[0]), __int_as_float(q[1]));
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
// Two sums in one pass (one barrier pair instead of two). scratch: 2*nwaves floats.
__device__ __forceinline__ float2 block_sum2(float2 v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v.x = wave_sum(v.x);
  v.y = wave_sum(v.y);
  __syncthreads();
  if (lane == 0) {
    scratch[2 * wid] = v.x;
    scratch[2 * wid + 1] = v.y;
  }
  __syncthreads();
  float2 r = make_float2(0.f, 0.f);
  for (int i = 0; i < nw; ++i) {
    r.x += scratch[2 * i];
    r.y += scratch[2 * i + 1];
  }
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
