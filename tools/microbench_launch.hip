// Microbenchmark: what does one tiny (1-workgroup) kernel cost inside a hipGraph on MI355X?
// Calibrates the fused DDP step's latency budget: per-node floor, per dependent global
// round trip, per KB of executed code (cold instruction cache), and LDS-only compute.
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench_launch.hip -o build/microbench_launch
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

__global__ void k_empty(int* p) {
  if (threadIdx.x == 0 && p[0] == 12345) p[1] = 1;
}

// `trips` dependent global loads (pointer chasing through a small table)
__global__ void k_chase(const int* tab, int* out, int trips) {
  int i = threadIdx.x & 63;
  for (int t = 0; t < trips; ++t) i = tab[i];
  if (threadIdx.x == 0) out[0] = i;
}

// straight-line code of N copies of an FMA block (forces I-cache footprint)
template <int N>
__global__ void k_code(float* out, float a) {
  float x = threadIdx.x * 1e-3f;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    x = fmaf(x, a, 0.5f);
    asm volatile("" : "+v"(x));
  }
  if (threadIdx.x == 0) out[0] = x;
}

// LDS-bound work like the fused step's phases: `rounds` dependent LDS passes with barriers
__global__ void k_lds(float* out, int rounds) {
  __shared__ float s[1024];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  float acc = 0.f;
  for (int r = 0; r < rounds; ++r) {
    acc += s[(threadIdx.x * 7 + r) & 1023];
    __syncthreads();
    s[threadIdx.x] = acc;
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = acc;
}

template <typename F>
double time_graph(hipStream_t st, int nodes, int reps, F launch) {
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < nodes; ++i) launch(st);
  hipStreamEndCapture(st, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, st);
  hipStreamSynchronize(st);
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) hipGraphLaunch(ge, st);
  hipStreamSynchronize(st);
  auto t1 = std::chrono::steady_clock::now();
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  return std::chrono::duration<double, std::micro>(t1 - t0).count() / (double(nodes) * reps);
}

int main() {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  int *tab, *out;
  float* fo;
  CK(hipMalloc(&tab, 64 * sizeof(int)));
  CK(hipMalloc(&out, 64 * sizeof(int)));
  CK(hipMalloc(&fo, 64 * sizeof(float)));
  std::vector<int> h(64);
  for (int i = 0; i < 64; ++i) h[i] = (i * 17 + 5) & 63;
  CK(hipMemcpy(tab, h.data(), 64 * sizeof(int), hipMemcpyHostToDevice));
  const int nodes = 200, reps = 20;
  std::printf("per-node time inside a %d-node hipGraph (us)\n", nodes);
  for (int thr : {64, 256, 1024})
    std::printf("empty kernel, 1 WG x %4d threads : %.2f\n", thr,
                time_graph(st, nodes, reps, [&](hipStream_t s) { hipLaunchKernelGGL(k_empty, 1, thr, 0, s, out); }));
  for (int trips : {1, 2, 4, 8})
    std::printf("dependent global loads x%d (L2-hot)  : %.2f\n", trips,
                time_graph(st, nodes, reps,
                           [&](hipStream_t s) { hipLaunchKernelGGL(k_chase, 1, 256, 0, s, tab, out, trips); }));
  std::printf("straight-line code   ~1 KB         : %.2f\n",
              time_graph(st, nodes, reps, [&](hipStream_t s) { hipLaunchKernelGGL(k_code<128>, 1, 256, 0, s, fo, 1.0001f); }));
  std::printf("straight-line code   ~8 KB         : %.2f\n",
              time_graph(st, nodes, reps, [&](hipStream_t s) { hipLaunchKernelGGL(k_code<1024>, 1, 256, 0, s, fo, 1.0001f); }));
  std::printf("straight-line code  ~32 KB         : %.2f\n",
              time_graph(st, nodes, reps, [&](hipStream_t s) { hipLaunchKernelGGL(k_code<4096>, 1, 256, 0, s, fo, 1.0001f); }));
  for (int r : {4, 16, 64})
    std::printf("LDS rounds x%-3d (2 barriers each)  : %.2f\n", r,
                time_graph(st, nodes, reps, [&](hipStream_t s) { hipLaunchKernelGGL(k_lds, 1, 1024, 0, s, fo, r); }));
  // alternate two different kernels (different code) back to back
  std::printf("alternating empty/code-8KB pairs   : %.2f\n",
              time_graph(st, nodes, reps, [&](hipStream_t s) {
                static int i = 0;
                if ((i++) & 1) hipLaunchKernelGGL(k_code<1024>, 1, 256, 0, s, fo, 1.0001f);
                else hipLaunchKernelGGL(k_empty, 1, 256, 0, s, out);
              }));
  return 0;
}
