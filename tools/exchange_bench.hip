// Microbenchmark: the single-wave engine's per-step gradient exchange in isolation.
// `world` workgroups of one wave each play the ranks of one GPU (each its own region of
// one uncached LL buffer, as XgmiComm allocates it); every iteration a dependent chain
// of `work` FMAs stands for the step's forward/loss/backward, then the layout-F chunk
// (KP = 5 weights + bias per lane, Linear(20, 1)) is exchanged and summed over the row
// slots (row16_sum), and the sum feeds the next iteration -- the engine's critical path.
// Variants: 0 = ll_exchange (round-2 protocol), 1 = ll_exchange_u (uniform poll loop,
// two batches in flight). Prints cycles (s_memtime) per iteration and checks that every
// rank ends with identical bits.
// Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -Icsrc tools/exchange_bench.hip -o tools/bin/exchange_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "kernels/linear_wave_impl.h"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

using namespace ptdt;
constexpr int KP = 5, DOUT = 1, DIN = 20;

template <int VARIANT>
__global__ void __launch_bounds__(64) k_exchange(uint64_t* buf, int world, int max_elems, int iters, int work,
                                                 int* err, long long* cycles, float* out) {
  const int rank = blockIdx.x;
  const int lane = threadIdx.x, q = lane >> 4, i = lane & 15, k0 = q * KP;
  const int64_t region = (int64_t)2 * world * max_elems;
  uint64_t PTDT_GLOBAL* const local = (uint64_t PTDT_GLOBAL*)(buf + rank * region);
  uint64_t PTDT_GLOBAL* push_dst = nullptr;
#pragma unroll
  for (int r = 0; r < kXgmiMaxRanks; ++r)
    if (i == r && r < world) push_dst = (uint64_t PTDT_GLOBAL*)(buf + r * region);
  float x = 1.f + 0.001f * (float)lane + 0.01f * (float)rank;
  float W[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) W[k] = 0.1f * (float)(k0 + k);
  uint32_t seq = 0;
  bool failed = false;
  const long long t0 = (long long)__builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters && !failed; ++it) {
    // the step's compute: a dependent chain on this lane's chunk
    float acc = x;
    for (int w = 0; w < work; ++w) acc = fmaf(acc, 0.999f, W[0] * 1e-3f);
    float gW[DOUT][KP], gb[DOUT];
#pragma unroll
    for (int k = 0; k < KP; ++k) gW[0][k] = lw::row16_sum(acc * (float)(k + 1) * 1e-3f);
    gb[0] = lw::row16_sum(acc * 1e-3f);
    if (world > 1) {
      seq += 1u;
      float v[DOUT][KP], vb[DOUT];
      bool ok;
      if constexpr (VARIANT == 0) {
#pragma unroll
        for (int k = 0; k < KP; ++k) v[0][k] = i == rank ? gW[0][k] : 0.f;
        vb[0] = i == rank ? gb[0] : 0.f;
        ok = lw::ll_exchange<KP, DOUT>(i < world && i != rank, push_dst, local, rank, i, world, max_elems, seq, k0,
                                       DIN, true, q == 0, false, gW, gb, v, vb, err, 1u << 20, false);
      } else {
        ok = lw::ll_exchange_u<KP, DOUT>(i < world && i != rank, push_dst, local, rank, i, world, max_elems, seq, k0,
                                         DIN, true, q == 0, false, gW, gb, v, vb, err, 1u << 20);
      }
      failed = __any(!ok);
#pragma unroll
      for (int k = 0; k < KP; ++k) gW[0][k] = lw::row16_sum(v[0][k]) * (1.f / (float)world);
      gb[0] = lw::row16_sum(vb[0]) * (1.f / (float)world);
    }
#pragma unroll
    for (int k = 0; k < KP; ++k) W[k] = fmaf(-0.01f, gW[0][k], W[k]);
    x = fmaf(-0.01f, gb[0], x);
  }
  const long long t1 = (long long)__builtin_amdgcn_s_memtime();
  if (lane == 0) cycles[rank] = t1 - t0;
#pragma unroll
  for (int k = 0; k < KP; ++k) out[(rank * 64 + lane) * (KP + 1) + k] = W[k];
  out[(rank * 64 + lane) * (KP + 1) + KP] = x;
}

template <int V>
int run(uint64_t* buf, int world, int max_elems, int iters, int work, int* err, long long* cyc, float* out) {
  CK(hipMemset(buf, 0, (size_t)8 * world * 2 * world * max_elems));
  CK(hipMemset(err, 0, sizeof(int)));
  hipLaunchKernelGGL((k_exchange<V>), dim3(world), dim3(64), 0, 0, buf, world, max_elems, iters, work, err, cyc, out);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  int e = 0;
  std::vector<long long> c(world);
  std::vector<float> o((size_t)world * 64 * (KP + 1));
  CK(hipMemcpy(&e, err, sizeof(int), hipMemcpyDeviceToHost));
  CK(hipMemcpy(c.data(), cyc, sizeof(long long) * world, hipMemcpyDeviceToHost));
  CK(hipMemcpy(o.data(), out, o.size() * sizeof(float), hipMemcpyDeviceToHost));
  // every rank's lanes of DPP row q hold chunk q: compare rank r's lanes against rank 0's
  // (ranks start from different x, so agreement needs the all-reduce to work)
  bool same = true;
  for (int r = 1; r < world; ++r)
    same &= std::memcmp(o.data(), o.data() + (size_t)r * 64 * (KP + 1), 64 * KP * sizeof(float)) == 0;
  long long mx = 0;
  for (long long v : c) mx = v > mx ? v : mx;
  std::printf("{\"variant\": %d, \"world\": %d, \"work\": %d, \"cycles_per_step\": %.1f, \"replicas_identical\": %s, "
              "\"err\": %d}\n",
              V, world, work, (double)mx / iters, same ? "true" : "false", e);
  return 0;
}

int main() {
  const int max_elems = 64, iters = 20000;
  uint64_t* buf;
  int* err;
  long long* cyc;
  float* out;
  CK(hipExtMallocWithFlags((void**)&buf, (size_t)8 * 8 * 2 * 8 * max_elems, hipDeviceMallocUncached));
  CK(hipMalloc(&err, sizeof(int)));
  CK(hipMalloc(&cyc, sizeof(long long) * 8));
  CK(hipMalloc(&out, sizeof(float) * 8 * 64 * (KP + 1)));
  for (int work : {0, 64}) {
    if (run<0>(buf, 1, max_elems, iters, work, err, cyc, out)) return 1;
    for (int world : {2, 4, 8}) {
      if (run<0>(buf, world, max_elems, iters, work, err, cyc, out)) return 1;
      if (run<1>(buf, world, max_elems, iters, work, err, cyc, out)) return 1;
    }
  }
  return 0;
}
