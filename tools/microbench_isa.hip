// Microbenchmark: issue cost (8 independent chains) and dependent latency (1 chain) of
// the wave-level instructions the single-wave engine (csrc/kernels/linear_wave_impl.h)
// is built from, in shader-clock cycles (s_memtime) on one wave of gfx950.
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench_isa.hip -o tools/bin/microbench_isa
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

enum Op { kFma, kDppRor8, kDppXor1, kSwap16, kSwap32, kPkFma, kDsRoundTrip, kSwizzle, kBpermute, kExp, kNumOps };
static const char* kNames[] = {"v_fma_f32", "v_add_f32_dpp row_ror:8", "v_add_f32_dpp quad_perm xor1",
                               "v_permlane16_swap+add", "v_permlane32_swap+add", "v_pk_fma_f32",
                               "ds_write+ds_read", "ds_swizzle(swap16)+add", "ds_bpermute+add", "v_exp_f32"};

template <int OP>
__device__ __forceinline__ float apply(float v, float* lds, int lane) {
  if constexpr (OP == kFma) {
    return fmaf(v, 1.0001f, 0.5f);
  } else if constexpr (OP == kDppRor8) {
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false));
  } else if constexpr (OP == kDppXor1) {
    return v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
  } else if constexpr (OP == kSwap16) {
    auto p = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
    return __int_as_float(p[0]) + __int_as_float(p[1]);
  } else if constexpr (OP == kSwap32) {
    auto p = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
    return __int_as_float(p[0]) + __int_as_float(p[1]);
  } else if constexpr (OP == kDsRoundTrip) {
    lds[lane] = v;
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    return lds[lane ^ 1] + 1.f;
  } else if constexpr (OP == kSwizzle) {
    // swizzle pattern: xor 16 over 32 lanes (bitmask mode: and 0x1f, xor 0x10)
    const int s = __builtin_amdgcn_ds_swizzle(__float_as_int(v), (0x10 << 10) | 0x1f);
    return v + __int_as_float(s);
  } else if constexpr (OP == kBpermute) {
    return v + __int_as_float(__builtin_amdgcn_ds_bpermute(((lane ^ 16) << 2), __float_as_int(v)));
  } else {
    return __expf(v) * 0.5f;
  }
}

template <int OP, int CH>
__global__ void __launch_bounds__(64) k_op(float* out, long long* cyc, int iters) {
  __shared__ float lds[64 * 8];
  const int lane = threadIdx.x;
  float v[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) v[c] = lane * 1e-3f + c;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {  // 16 x CH ops per loop trip: loop overhead amortised
    if constexpr (OP == kPkFma) {
#pragma unroll
      for (int c = 0; c + 1 < CH || c == 0; c += 2) {
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 a = {v[c], CH > 1 ? v[c + 1] : v[c]};
        const f2 m = {1.0001f, 1.0001f}, b = {0.5f, 0.5f};
        a = __builtin_elementwise_fma(a, m, b);
        v[c] = a.x;
        if (CH > 1) v[c + 1] = a.y;
      }
    } else {
#pragma unroll
      for (int c = 0; c < CH; ++c) v[c] = apply<OP>(v[c], lds + 64 * c, lane);
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) asm volatile("" : "+v"(v[c]));
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += v[c];
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[lane] = s;
  if (lane == 0) cyc[0] = t1 - t0;
}

// L2-hit latency: dependent loads through a 64-entry table
__global__ void __launch_bounds__(64) k_chase(const int* tab, int* out, long long* cyc, int iters) {
  int i = threadIdx.x;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int t = 0; t < iters; ++t) i = tab[i];
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = i;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// dependent system-scope (L2-bypassing) loads, as the all-reduce polls issue them
__global__ void __launch_bounds__(64) k_chase_sys(int* tab, int* out, long long* cyc, int iters) {
  int i = threadIdx.x;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int t = 0; t < iters; ++t) i = __hip_atomic_load(tab + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = i;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// store a new value, spin until a system-scope load returns it
__global__ void __launch_bounds__(64) k_store_visible(int* buf, long long* cyc, int iters) {
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int t = 1; t <= iters; ++t) {
    __hip_atomic_store(buf + threadIdx.x, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    int spins = 0;
    while (__hip_atomic_load(buf + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != t && ++spins < 100000) {
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int OP>
int run_op(float* out, long long* dcyc) {
  const int iters = 1024;
  long long c1 = 0, c8 = 0;
  for (int rep = 0; rep < 2; ++rep) {  // second run: warm I-cache
    hipLaunchKernelGGL((k_op<OP, 1>), dim3(1), dim3(64), 0, 0, out, dcyc, iters);
    CK(hipMemcpy(&c1, dcyc, 8, hipMemcpyDeviceToHost));
    hipLaunchKernelGGL((k_op<OP, 8>), dim3(1), dim3(64), 0, 0, out, dcyc, iters);
    CK(hipMemcpy(&c8, dcyc, 8, hipMemcpyDeviceToHost));
  }
  std::printf("%-32s latency %6.2f  issue %6.2f cycles\n", kNames[OP], (double)c1 / (16.0 * iters),
              (double)c8 / (8.0 * 16.0 * iters));
  return 0;
}

int main() {
  float* out;
  long long* dcyc;
  int *tab, *iout;
  CK(hipMalloc(&out, 64 * sizeof(float)));
  CK(hipMalloc(&dcyc, sizeof(long long)));
  CK(hipMalloc(&tab, 64 * sizeof(int)));
  CK(hipMalloc(&iout, 64 * sizeof(int)));
  int h[64];
  for (int i = 0; i < 64; ++i) h[i] = (i * 17 + 5) & 63;
  CK(hipMemcpy(tab, h, sizeof(h), hipMemcpyHostToDevice));
  if (run_op<kFma>(out, dcyc) || run_op<kDppRor8>(out, dcyc) || run_op<kDppXor1>(out, dcyc) ||
      run_op<kSwap16>(out, dcyc) || run_op<kSwap32>(out, dcyc) || run_op<kPkFma>(out, dcyc) ||
      run_op<kDsRoundTrip>(out, dcyc) || run_op<kSwizzle>(out, dcyc) || run_op<kBpermute>(out, dcyc) ||
      run_op<kExp>(out, dcyc))
    return 1;
  long long c = 0;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, tab, iout, dcyc, 2048);
    CK(hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost));
  }
  std::printf("%-32s latency %6.2f cycles\n", "global_load (L1 hit, 256 B table)", (double)c / 2048);
  // 1 MiB table, 4 KiB stride walk: misses L1 (32 KiB), hits L2 (4 MiB per XCD) after the first lap
  const int n = 1 << 18;
  int* big;
  CK(hipMalloc(&big, n * sizeof(int)));
  int* hb = new int[n];
  for (int i = 0; i < n; ++i) hb[i] = (i + 1024 + 64 * ((i >> 10) & 7)) % n;
  CK(hipMemcpy(big, hb, n * sizeof(int), hipMemcpyHostToDevice));
  delete[] hb;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, big, iout, dcyc, 4096);
    CK(hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost));
  }
  std::printf("%-32s latency %6.2f cycles\n", "global_load (L2 hit, 1 MiB walk)", (double)c / 4096);
  // polling memory of the one-shot all-reduce: uncached and fine-grained allocations
  // (64-entry table, so a cacheable allocation would hit L1)
  for (int kind = 0; kind < 2; ++kind) {
    int* t2;
    CK(hipExtMallocWithFlags((void**)&t2, 64 * sizeof(int),
                             kind == 0 ? hipDeviceMallocUncached : hipDeviceMallocFinegrained));
    CK(hipMemcpy(t2, h, sizeof(h), hipMemcpyHostToDevice));
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(k_chase_sys, dim3(1), dim3(64), 0, 0, t2, iout, dcyc, 1024);
      CK(hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost));
    }
    std::printf("%-32s latency %6.2f cycles\n", kind == 0 ? "system-scope load, uncached mem" : "system-scope load, fine-grained",
                (double)c / 1024);
    CK(hipFree(t2));
  }
  {  // store -> visible to a system-scope load of the same wave (write round trip on uncached memory)
    int* t3;
    CK(hipExtMallocWithFlags((void**)&t3, 64 * sizeof(int), hipDeviceMallocUncached));
    CK(hipMemset(t3, 0, 64 * sizeof(int)));
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(k_store_visible, dim3(1), dim3(64), 0, 0, t3, dcyc, 1024);
      CK(hipMemcpy(&c, dcyc, 8, hipMemcpyDeviceToHost));
    }
    std::printf("%-32s latency %6.2f cycles\n", "store->load seen, uncached mem", (double)c / 1024);
    CK(hipFree(t3));
  }
  CK(hipDeviceSynchronize());
  return 0;
}
