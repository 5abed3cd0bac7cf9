// On-device synthetic data (gfx950): Philox4x32-10 counter RNG, one-hot
// labels and batch row gather.
//
// Replaces the reference's CPU-side synthetic data + per-step H2D copies
// (ddp_gpus.py:61 torch.rand, NB01:121 torch.randn, NB03:958,984 randn + one-hot
// scatter_ then .to(cuda)): data is generated where it is
// consumed, so no PCIe traffic sits in the step.
#include "common.h"
#include "kernels.h"
#include "sampler.h"

namespace ptdt {
namespace {

constexpr int kBlock = 256;

struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox4x32_10(U4 ctr, uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    const uint32_t hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    ctr = U4{hi1 ^ ctr.y ^ k0, lo1, hi0 ^ ctr.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return ctr;
}

// uniform in [0, 1) with 24 random mantissa bits (never returns 1.0)
__device__ __forceinline__ float u01(uint32_t v) { return (float)(v >> 8) * (1.0f / 16777216.0f); }

__global__ void __launch_bounds__(kBlock) philox_kernel(float* out, int64_t n, uint32_t k0, uint32_t k1,
                                                        uint64_t offset, int dist) {
  const int64_t nq = (n + 3) / 4;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < nq; q += stride) {
    const uint64_t c = offset + (uint64_t)q;
    const U4 r = philox4x32_10(U4{(uint32_t)c, (uint32_t)(c >> 32), 0u, 0u}, k0, k1);
    float v[4];
    if (dist == 0) {
      v[0] = u01(r.x); v[1] = u01(r.y); v[2] = u01(r.z); v[3] = u01(r.w);
    } else {
      // Box-Muller on two pairs; 1 - u keeps the log argument in (0, 1]
      const float r0 = sqrtf(-2.f * logf(1.f - u01(r.x))), t0 = 6.2831853071795864f * u01(r.y);
      const float r1 = sqrtf(-2.f * logf(1.f - u01(r.z))), t1 = 6.2831853071795864f * u01(r.w);
      float s0, c0, s1, c1;
      sincosf(t0, &s0, &c0);
      sincosf(t1, &s1, &c1);
      v[0] = r0 * c0; v[1] = r0 * s0; v[2] = r1 * c1; v[3] = r1 * s1;
    }
    const int64_t base = 4 * q;
    if (base + 3 < n && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
      reinterpret_cast<float4*>(out)[q] = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      for (int j = 0; j < 4 && base + j < n; ++j) out[base + j] = v[j];
    }
  }
}

__global__ void __launch_bounds__(kBlock) one_hot_kernel(const int64_t* idx, float* out, int B, int C) {
  const int64_t n = (int64_t)B * C;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x; e < n; e += stride) {
    const int b = (int)(e / C), c = (int)(e % C);
    out[e] = (idx[b] == c) ? 1.f : 0.f;
  }
}

// One workgroup row-tile; 4-byte words when the row is word aligned.
__global__ void __launch_bounds__(kBlock) gather_rows_kernel(const uint8_t* src, const int32_t* idx,
                                                             uint8_t* out, int64_t rows,
                                                             int64_t row_bytes) {
  const bool words = (row_bytes & 3) == 0;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const uint8_t* s = src + (int64_t)idx[r] * row_bytes;
    uint8_t* d = out + r * row_bytes;
    if (words) {
      for (int64_t i = threadIdx.x; i < row_bytes / 4; i += kBlock)
        reinterpret_cast<uint32_t*>(d)[i] = reinterpret_cast<const uint32_t*>(s)[i];
    } else {
      for (int64_t i = threadIdx.x; i < row_bytes; i += kBlock) d[i] = s[i];
    }
  }
}

// ---- device DistributedSampler (csrc/kernels/sampler.h)
__global__ void __launch_bounds__(1024) sampler_kernel(int32_t* out, int64_t N, int W, int rank,
                                                       int64_t num_samples, uint64_t seed,
                                                       int32_t* epoch_ptr, int shuffle) {
  const int epoch = *epoch_ptr + 1;
  rank_epoch_indices(out, (uint32_t)N, W, rank, (int)num_samples, seed, epoch, shuffle, threadIdx.x, blockDim.x);
  __syncthreads();
  if (threadIdx.x == 0) *epoch_ptr = epoch;
}

}  // namespace

hipError_t device_sampler(int32_t* out, int64_t N, int W, int rank, int64_t num_samples, uint64_t seed,
                          int32_t* epoch_ptr, int shuffle, hipStream_t s) {
  if (N <= 0 || N > (1ll << 30) || W <= 0 || rank < 0 || rank >= W) return hipErrorInvalidValue;
  // one workgroup: it reads the epoch, writes all indices, then publishes the
  // new epoch after a barrier (no cross-workgroup race on the counter)
  hipLaunchKernelGGL(sampler_kernel, dim3(1), dim3(1024), 0, s, out, N, W, rank, num_samples, seed,
                     epoch_ptr, shuffle);
  return hipGetLastError();
}

hipError_t philox_fill(float* out, int64_t n, uint64_t seed, uint64_t offset, int dist, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t nq = (n + 3) / 4;
  int64_t g = (nq + kBlock - 1) / kBlock;
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(philox_kernel, dim3((int)g), dim3(kBlock), 0, s, out, n, (uint32_t)seed,
                     (uint32_t)(seed >> 32), offset, dist);
  return hipGetLastError();
}

hipError_t one_hot(const int64_t* idx, float* out, int B, int C, hipStream_t s) {
  const int64_t n = (int64_t)B * C;
  if (n <= 0) return hipSuccess;
  int64_t g = (n + kBlock - 1) / kBlock;
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(one_hot_kernel, dim3((int)g), dim3(kBlock), 0, s, idx, out, B, C);
  return hipGetLastError();
}

hipError_t gather_rows(const void* src, const int32_t* idx, void* out, int64_t rows, int64_t cols,
                       int elem_bytes, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  const int g = (int)(rows < 2048 ? rows : 2048);
  hipLaunchKernelGGL(gather_rows_kernel, dim3(g), dim3(kBlock), 0, s, (const uint8_t*)src, idx,
                     (uint8_t*)out, rows, cols * elem_bytes);
  return hipGetLastError();
}

}  // namespace ptdt
