// Host <-> device clock calibration for launch timelines (tools/driver_timeline.py).
//
// The persistent engines can stamp the 100 MHz realtime counter at fixed points of a
// launch (PersistArgs::tl). To place those stamps on the host's CLOCK_MONOTONIC axis
// next to the host's own stamps (before/after hipLaunchKernel, after the synchronize),
// one single-thread kernel answers n pings: the host stores flag[k] = k + 1 into
// host-mapped memory and notes the time, the kernel sees it, stores its realtime counter
// into out[k] (host-mapped), and the host notes when that answer arrives. Each ping
// bounds the offset between the clocks by its round trip; the tightest pings win.
// The kernel's poll loop is bounded (kMaxPolls per ping), so it always drains.
#include <time.h>

#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

constexpr uint32_t kMaxPolls = 1u << 22;  // ~1 s of polling per ping at most

__global__ void clock_ping_kernel(const int32_t* flag, int64_t* out, int n) {
  for (int k = 0; k < n; ++k) {
    bool seen = false;
    for (uint32_t p = 0; p < kMaxPolls; ++p) {
      if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == k + 1) {
        seen = true;
        break;
      }
    }
    const int64_t t = seen ? (int64_t)__builtin_amdgcn_s_memrealtime() : -1;
    __hip_atomic_store(out + k, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (!seen) return;  // the host gave up: stop answering
  }
}

int64_t now_ns() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (int64_t)t.tv_sec * 1000000000 + t.tv_nsec;
}

}  // namespace

hipError_t clock_calibrate(int n, int64_t* host_set, int64_t* host_seen, int64_t* dev_ticks) {
  if (n <= 0 || n > 4096) return hipErrorInvalidValue;
  int32_t* flag = nullptr;
  int64_t* out = nullptr;
  PTDT_HIP_CHECK(hipHostMalloc((void**)&flag, sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent));
  hipError_t err = hipHostMalloc((void**)&out, n * sizeof(int64_t), hipHostMallocMapped | hipHostMallocCoherent);
  if (err != hipSuccess) {
    hipHostFree(flag);
    return err;
  }
  volatile int32_t* vf = flag;
  volatile int64_t* vo = out;
  *vf = 0;
  for (int k = 0; k < n; ++k) vo[k] = 0;
  int32_t* dflag = nullptr;
  int64_t* dout = nullptr;
  err = hipHostGetDevicePointer((void**)&dflag, flag, 0);
  if (err == hipSuccess) err = hipHostGetDevicePointer((void**)&dout, out, 0);
  hipStream_t s = nullptr;
  if (err == hipSuccess) err = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (err == hipSuccess) {
    hipLaunchKernelGGL(clock_ping_kernel, dim3(1), dim3(1), 0, s, dflag, dout, n);
    err = hipGetLastError();
  }
  if (err == hipSuccess) {
    const int64_t t_start = now_ns();
    for (int k = 0; k < n; ++k) {
      // let the kernel get going first; pings are spaced so each one is a fresh round trip
      const int64_t t_next = now_ns() + (k == 0 ? 2000000 : 20000);
      while (now_ns() < t_next) {
      }
      host_set[k] = now_ns();
      __atomic_store_n(flag, k + 1, __ATOMIC_SEQ_CST);
      int64_t v = 0;
      for (;;) {
        v = vo[k];
        if (v != 0) break;
        if (now_ns() - t_start > 2000000000ll) break;  // 2 s: give up (the kernel stops too)
      }
      host_seen[k] = now_ns();
      dev_ticks[k] = v;
      if (v <= 0) {
        for (int j = k; j < n; ++j) dev_ticks[j] = -1;
        break;
      }
    }
    const hipError_t e2 = hipStreamSynchronize(s);
    if (err == hipSuccess) err = e2;
  }
  if (s) hipStreamDestroy(s);
  hipHostFree(out);
  hipHostFree(flag);
  return err;
}

}  // namespace ptdt
