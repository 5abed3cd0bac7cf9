// Standalone one-shot xGMI all-reduce (average) for small fp32 buckets.
// Protocol and safety notes: csrc/comm/xgmi.h.
#include "../comm/xgmi.h"
#include "common.h"

namespace ptdt {
namespace {

__global__ void __launch_bounds__(1024) xgmi_ar_kernel(XgmiArgs x, float* data, int n) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const uint32_t s = *x.seq + 1u;
  xgmi_push(x, s, data, n, tid, nt);
  __syncthreads();  // every read of `data` precedes the first overwrite
  const float inv = 1.f / (float)x.world;
  for (int i = tid; i < n; i += nt) data[i] = xgmi_gather_sum(x, s, i) * inv;
  __syncthreads();
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
