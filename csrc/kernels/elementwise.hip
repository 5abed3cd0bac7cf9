// Elementwise / reduction helpers (gfx950), all grid-stride with capped grids
// (<= 2048 workgroups = 256 CUs x 8) and 16-byte vector accesses on the fp32
// fast paths.
#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

constexpr int kBlock = 256;

inline int grid_for(int64_t n, int per_thread = 4) {
  int64_t g = (n + (int64_t)kBlock * per_thread - 1) / ((int64_t)kBlock * per_thread);
  return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

template <typename T>
__global__ void __launch_bounds__(kBlock) relu_bwd_kernel(const T* dy, const T* y, T* dx, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    Cvt<T>::store(dx, i, Cvt<T>::load(y, i) > 0.f ? Cvt<T>::load(dy, i) : 0.f);
}

// out[c] (+)= sum_r x[r, c] in a FIXED order (no atomics, no memset: bit-identical
// across launches, and nothing in it depends on a memset node when it is replayed
// from a hipGraph -- a captured hipMemsetAsync was seen to zero only part of the
// buffer once eager memsets had run between replays, profiles/r4_graph_memset.md).
// A workgroup (4 waves) owns 64 columns (one per lane) and a row range; wave w sums
// rows w, w+4, ...; the 4 partials meet in LDS in wave order. With nsplit > 1 the
// row ranges write partials to ws[split][cols] and col_sum_finish adds them in order.
template <typename T>
__global__ void __launch_bounds__(kBlock) col_sum_kernel(const T* x, int64_t rows, int64_t cols, float* out,
                                                         float* ws, int64_t rows_per, int accumulate) {
  __shared__ float red[kBlock / 64][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + lane;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per;
  const int64_t r1 = min(rows, r0 + rows_per);
  float s = 0.f;
  if (c < cols)
    for (int64_t r = r0 + w; r < r1; r += kBlock / 64) s += Cvt<T>::load(x, r * cols + c);
  red[w][lane] = s;
  __syncthreads();
  if (w != 0 || c >= cols) return;
  s = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
  if (ws != nullptr)
    ws[(int64_t)blockIdx.y * cols + c] = s;
  else
    out[c] = accumulate ? out[c] + s : s;
}

__global__ void __launch_bounds__(kBlock) col_sum_finish_kernel(const float* ws, int nsplit, int64_t cols, float* out,
                                                                int accumulate) {
  const int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
  for (int k = 0; k < nsplit; ++k) s += ws[(int64_t)k * cols + c];
  out[c] = accumulate ? out[c] + s : s;
}

// Sum of all elements into out[0] (fp32 accumulation, fixed order: deterministic).
// One workgroup: the DP toy loss reduces [32, 2] (NB01:485); larger
// inputs still run in one pass, 4 independent accumulators per thread.
template <typename T>
__global__ void __launch_bounds__(kBlock) sum_all_kernel(const T* x, int64_t n, float* out) {
  __shared__ float scratch[kBlock / 64];
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int64_t i = threadIdx.x;
  for (; i + 3 * kBlock < n; i += 4 * kBlock) {
    a0 += Cvt<T>::load(x, i);
    a1 += Cvt<T>::load(x, i + kBlock);
    a2 += Cvt<T>::load(x, i + 2 * kBlock);
    a3 += Cvt<T>::load(x, i + 3 * kBlock);
  }
  for (; i < n; i += kBlock) a0 += Cvt<T>::load(x, i);
  const float s = block_sum((a0 + a1) + (a2 + a3), scratch);
  if (threadIdx.x == 0) out[0] = s;
}

__global__ void __launch_bounds__(kBlock) fill_kernel(float* x, float v, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) x[i] = v;
}

__global__ void __launch_bounds__(kBlock) f32_to_bf16_kernel(const float* x, uint16_t* y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) y[i] = f32_to_bf16(x[i]);
}
__global__ void __launch_bounds__(kBlock) bf16_to_f32_kernel(const uint16_t* x, float* y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) y[i] = bf16_to_f32(x[i]);
}

// y = relu?(x * scale[c] + shift[c]) over NCHW (flat grid-stride, c = (i / HW) % C).
template <typename T>
__global__ void __launch_bounds__(kBlock) bn_relu_kernel(const T* x, const float* scale,
                                                         const float* shift, int64_t n, int64_t C,
                                                         int64_t HW, int relu, T* y) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const int c = (int)((i / HW) % C);
    float v = fmaf(Cvt<T>::load(x, i), scale[c], shift[c]);
    if (relu) v = fmaxf(v, 0.f);
    Cvt<T>::store(y, i, v);
  }
}

}  // namespace

// NHWC 3-channel pixels (f32 or bf16) -> NHWC 4-channel bf16 with a zero 4th channel: the RGB stem's
// input for the 4-channel convolution (ops/conv.py), cast and padded in one pass (8 B stored per pixel).
template <typename T>
__global__ void __launch_bounds__(kBlock) rgb4_pack_kernel(const T* __restrict__ x, uint2* __restrict__ y, int64_t npix) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < npix; p += stride) {
    const T* px = x + 3 * p;
    const uint32_t r = f32_to_bf16(Cvt<T>::load(px, 0)), g = f32_to_bf16(Cvt<T>::load(px, 1)),
                   b = f32_to_bf16(Cvt<T>::load(px, 2));
    y[p] = make_uint2(r | (g << 16), b);
  }
}

hipError_t rgb4_pack(const void* x, int dtype, uint16_t* y, int64_t npix, hipStream_t s) {
  if (npix <= 0) return hipSuccess;
  int64_t blocks = (npix + kBlock - 1) / kBlock;
  if (blocks > 8192) blocks = 8192;
  if (dtype == kF32)
    hipLaunchKernelGGL(rgb4_pack_kernel<float>, dim3((int)blocks), dim3(kBlock), 0, s, static_cast<const float*>(x),
                       reinterpret_cast<uint2*>(y), npix);
  else
    hipLaunchKernelGGL(rgb4_pack_kernel<uint16_t>, dim3((int)blocks), dim3(kBlock), 0, s,
                       static_cast<const uint16_t*>(x), reinterpret_cast<uint2*>(y), npix);
  return hipGetLastError();
}

hipError_t relu_backward(const void* dy, const void* y, void* dx, int dtype, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (dtype == kF32)
    hipLaunchKernelGGL(relu_bwd_kernel<float>, dim3(grid_for(n)), dim3(kBlock), 0, s,
                       (const float*)dy, (const float*)y, (float*)dx, n);
  else
    hipLaunchKernelGGL(relu_bwd_kernel<uint16_t>, dim3(grid_for(n)), dim3(kBlock), 0, s,
                       (const uint16_t*)dy, (const uint16_t*)y, (uint16_t*)dx, n);
  return hipGetLastError();
}

int col_sum_splits(int64_t rows, int64_t cols) {
  const int64_t gx = (cols + 63) / 64;
  int64_t want = (256 + gx - 1) / gx;              // ~256 workgroups in flight
  const int64_t by_rows = (rows + 1023) / 1024;   // >= 1024 rows per split
  if (want > by_rows) want = by_rows;
  if (want > 64) want = 64;
  return want < 1 ? 1 : (int)want;
}

hipError_t col_sum(const void* x, int dtype, int64_t rows, int64_t cols, float* out, int accumulate, float* ws,
                   int nsplit, hipStream_t s) {
  if (cols <= 0) return hipSuccess;
  if (nsplit < 1 || (nsplit > 1 && ws == nullptr)) return hipErrorInvalidValue;
  if (rows < 0) rows = 0;
  const int64_t rows_per = nsplit > 1 ? (rows + nsplit - 1) / nsplit : (rows > 0 ? rows : 1);
  const dim3 grid((unsigned)((cols + 63) / 64), (unsigned)nsplit);
  float* part = nsplit > 1 ? ws : nullptr;
  if (dtype == kF32)
    hipLaunchKernelGGL(col_sum_kernel<float>, grid, dim3(kBlock), 0, s, (const float*)x, rows, cols, out, part,
                       rows_per, accumulate);
  else
    hipLaunchKernelGGL(col_sum_kernel<uint16_t>, grid, dim3(kBlock), 0, s, (const uint16_t*)x, rows, cols, out,
                       part, rows_per, accumulate);
  PTDT_HIP_CHECK(hipGetLastError());
  if (nsplit > 1)
    hipLaunchKernelGGL(col_sum_finish_kernel, dim3((unsigned)((cols + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, ws,
                       nsplit, cols, out, accumulate);
  return hipGetLastError();
}

hipError_t sum_all(const void* x, int dtype, int64_t n, float* out, hipStream_t s) {
  if (n <= 0) return hipErrorInvalidValue;
  if (dtype == kF32)
    hipLaunchKernelGGL(sum_all_kernel<float>, dim3(1), dim3(kBlock), 0, s, (const float*)x, n, out);
  else
    hipLaunchKernelGGL(sum_all_kernel<uint16_t>, dim3(1), dim3(kBlock), 0, s, (const uint16_t*)x, n, out);
  return hipGetLastError();
}

hipError_t fill_f32(float* x, float v, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, x, v, n);
  return hipGetLastError();
}

hipError_t cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, x, y, n);
  return hipGetLastError();
}

hipError_t cast_bf16_f32(const uint16_t* x, float* y, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(bf16_to_f32_kernel, dim3(grid_for(n)), dim3(kBlock), 0, s, x, y, n);
  return hipGetLastError();
}

hipError_t bn_relu_apply(const void* x, int dtype, const float* scale, const float* shift, int64_t N,
                         int64_t C, int64_t HW, int relu, void* y, hipStream_t s) {
  const int64_t n = N * C * HW;
  if (n <= 0) return hipSuccess;
  if (dtype == kF32)
    hipLaunchKernelGGL(bn_relu_kernel<float>, dim3(grid_for(n)), dim3(kBlock), 0, s, (const float*)x,
                       scale, shift, n, C, HW, relu, (float*)y);
  else
    hipLaunchKernelGGL(bn_relu_kernel<uint16_t>, dim3(grid_for(n)), dim3(kBlock), 0, s,
                       (const uint16_t*)x, scale, shift, n, C, HW, relu, (uint16_t*)y);
  return hipGetLastError();
}

// ------------------------------------------------------------ comm_done_mark
__global__ void comm_done_mark_kernel(unsigned long long* ctr, uint64_t* host_mirror) {
  const unsigned long long v = atomicAdd(ctr, 1ull) + 1ull;
  __hip_atomic_store(host_mirror, (uint64_t)v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t comm_done_mark(uint64_t* ctr, uint64_t* host_mirror, hipStream_t s) {
  hipLaunchKernelGGL(comm_done_mark_kernel, dim3(1), dim3(1), 0, s, reinterpret_cast<unsigned long long*>(ctr),
                     host_mirror);
  return hipGetLastError();
}

}  // namespace ptdt
