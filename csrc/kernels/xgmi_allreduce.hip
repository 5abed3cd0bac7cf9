// Standalone one-shot xGMI all-reduce (average) for small fp32 buckets.
// Protocol and safety notes: csrc/comm/xgmi.h.
#include "../comm/xgmi.h"
#include "common.h"

namespace ptdt {
namespace {

constexpr int kChunk = 2048;  // elements per staging pass: 8 ranks x 2048 x 4 B = 64 KiB LDS

__global__ void __launch_bounds__(1024) xgmi_ar_kernel(XgmiArgs x, float* data, int n) {
  __shared__ float tmp[kXgmiMaxRanks * kChunk];
  const int tid = threadIdx.x, nt = blockDim.x;
  const uint32_t s = *x.seq + 1u;
  xgmi_push(x, s, data, n, tid, nt);
  __syncthreads();  // every read of `data` precedes the first overwrite
  const float inv = 1.f / (float)x.world;
  for (int i0 = 0; i0 < n; i0 += kChunk) {
    const int m = n - i0 < kChunk ? n - i0 : kChunk;
    xgmi_gather_lds(x, s, i0, m, tmp, tid, nt);
    __syncthreads();
    for (int i = tid; i < m; i += nt) data[i0 + i] = xgmi_sum_lds(tmp, x.world, m, i) * inv;
    __syncthreads();
  }
  if (tid == 0) *x.seq = s;
}

}  // namespace

hipError_t xgmi_allreduce_avg(const XgmiArgs& x, float* data, int n, hipStream_t s) {
  if (x.world <= 0 || n < 0 || n > x.max_elems || x.world > kXgmiMaxRanks) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(xgmi_ar_kernel, dim3(1), dim3(1024), 0, s, x, data, n);
  return hipGetLastError();
}

}  // namespace ptdt
