// Microbenchmark: flag latency between two workgroups on one MI355X (the in-kernel
// all-reduce's exchange in isolation: a 64-bit LL word stored by one wave, polled by
// another). Ping-pong of `iters` round trips; reports cycles (s_memtime) per round trip
// for each memory type (uncached / fine-grained / coarse-grained), memory scope
// (system / agent), poll style (one load in flight + s_sleep, or P loads in flight,
// staggered) and placement (the two workgroups on different XCDs or on the same one).
// Polls are bounded (a lost word ends the kernel with err set, never a hang).
// Build: hipcc --offload-arch=gfx950 -O3 tools/pingpong.hip -o tools/bin/pingpong
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

constexpr uint32_t kMaxPolls = 1u << 20;

template <int SCOPE>
__device__ __forceinline__ uint64_t ld(uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, SCOPE);
}
template <int SCOPE>
__device__ __forceinline__ void st(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, SCOPE);
}

// wait until *p == want; P loads in flight (P == 1: load, check, s_sleep SLEEP)
template <int SCOPE, int P, int SLEEP>
__device__ __forceinline__ bool wait_eq(uint64_t* p, uint64_t want) {
  if constexpr (P == 1) {
    for (uint32_t n = 0; n < kMaxPolls; ++n) {
      if (ld<SCOPE>(p) == want) return true;
      if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
    }
    return false;
  } else {
    uint64_t w[P];
#pragma unroll
    for (int i = 0; i < P; ++i) {
      w[i] = ld<SCOPE>(p);
      if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
    }
    for (uint32_t n = 0; n < kMaxPolls; n += P) {
#pragma unroll
      for (int i = 0; i < P; ++i) {  // the oldest load first; reissue it as the youngest
        if (w[i] == want) return true;
        w[i] = ld<SCOPE>(p);
      }
    }
    return false;
  }
}

template <int SCOPE, int P, int SLEEP>
__global__ void k_pingpong(uint64_t* a, uint64_t* b, int iters, int pong_block, int* err, long long* cycles) {
  const int blk = blockIdx.x;
  if ((blk != 0 && blk != pong_block) || threadIdx.x != 0) return;
  const bool ping = blk == 0;
  uint64_t* mine = ping ? a : b;
  uint64_t* theirs = ping ? b : a;
  const long long t0 = (long long)__builtin_amdgcn_s_memtime();
  for (int k = 1; k <= iters; ++k) {
    if (ping) {
      st<SCOPE>(theirs, (uint64_t)k);
      if (!wait_eq<SCOPE, P, SLEEP>(mine, (uint64_t)k)) { *err = 1; break; }
    } else {
      if (!wait_eq<SCOPE, P, SLEEP>(mine, (uint64_t)k)) { *err = 1; break; }
      st<SCOPE>(theirs, (uint64_t)k);
    }
  }
  if (ping) *cycles = (long long)__builtin_amdgcn_s_memtime() - t0;
}

template <int SCOPE, int P, int SLEEP>
int run(const char* mem, uint64_t* a, uint64_t* b, int* err, long long* cyc, int pong_block, const char* where) {
  const int iters = 20000;
  CK(hipMemset(a, 0, 64));
  CK(hipMemset(b, 0, 64));
  CK(hipMemset(err, 0, sizeof(int)));
  hipLaunchKernelGGL((k_pingpong<SCOPE, P, SLEEP>), dim3(16), dim3(64), 0, 0, a, b, iters, pong_block, err, cyc);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  int e = 0;
  long long c = 0;
  CK(hipMemcpy(&e, err, sizeof(int), hipMemcpyDeviceToHost));
  CK(hipMemcpy(&c, cyc, sizeof(long long), hipMemcpyDeviceToHost));
  std::printf("{\"mem\": \"%s\", \"scope\": \"%s\", \"polls_in_flight\": %d, \"sleep\": %d, \"placement\": \"%s\", "
              "\"cycles_per_round_trip\": %.1f, \"err\": %d}\n",
              mem, SCOPE == __HIP_MEMORY_SCOPE_SYSTEM ? "system" : "agent", P, SLEEP, where, (double)c / iters, e);
  return 0;
}

template <int SCOPE>
int sweep(const char* mem, uint64_t* a, uint64_t* b, int* err, long long* cyc) {
  for (int pb : {1, 8}) {
    const char* where = pb == 1 ? "different XCDs (blocks 0, 1)" : "same XCD (blocks 0, 8)";
    if (run<SCOPE, 1, 1>(mem, a, b, err, cyc, pb, where)) return 1;
    if (run<SCOPE, 1, 0>(mem, a, b, err, cyc, pb, where)) return 1;
    if (run<SCOPE, 2, 0>(mem, a, b, err, cyc, pb, where)) return 1;
    if (run<SCOPE, 4, 0>(mem, a, b, err, cyc, pb, where)) return 1;
    if (run<SCOPE, 4, 2>(mem, a, b, err, cyc, pb, where)) return 1;
  }
  return 0;
}

int main() {
  int* err;
  long long* cyc;
  CK(hipMalloc(&err, sizeof(int)));
  CK(hipMalloc(&cyc, sizeof(long long)));
  struct M {
    const char* name;
    unsigned flags;
    bool plain;
  } mems[] = {{"uncached", hipDeviceMallocUncached, false},
              {"finegrained", hipDeviceMallocFinegrained, false},
              {"coarse", 0, true}};
  for (const M& m : mems) {
    void* buf = nullptr;
    if (m.plain) CK(hipMalloc(&buf, 4096));
    else CK(hipExtMallocWithFlags(&buf, 4096, m.flags));
    uint64_t* a = static_cast<uint64_t*>(buf);
    uint64_t* b = a + 256;  // separate 2 KiB: no shared cache line
    if (sweep<__HIP_MEMORY_SCOPE_SYSTEM>(m.name, a, b, err, cyc)) return 1;
    if (sweep<__HIP_MEMORY_SCOPE_AGENT>(m.name, a, b, err, cyc)) return 1;
    CK(hipFree(buf));
  }
  return 0;
}
