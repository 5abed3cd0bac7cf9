// Minimal reproducer: a hipMemsetAsync captured into a hipGraph, replayed after EAGER
// hipMemsetAsync calls on other buffers (no torch, no framework code).
//
// Observed through the framework (profiles/r4_graph_memset.md): the Linear bias-gradient column
// sum's captured zero-fill left part of its buffer unzeroed once eager steps (which issue their own
// memsets, e.g. MIOpen's atomic weight-gradient solvers) ran between replays. This program checks
// the runtime alone: per case it captures {memset(A, 0) ; kernel A += 1} on a stream, replays it once
// (A must be all 1), then runs `eager` eager memsets of a DIFFERENT buffer B (optionally of another
// size, on another stream), fills A with a sentinel, replays again and counts the words of A that
// are not 1.
//
//   hipcc --offload-arch=gfx950 -O2 tools/graph_memset_repro.hip -o build/graph_memset_repro
//   ./build/graph_memset_repro      # one line per case: bad words after each replay round
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                   \
    }                                                                                 \
  } while (0)

__global__ void add_one(float* a, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] += 1.f;
}

__global__ void fill(float* a, int n, float v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = v;
}

static int count_bad(const float* dA, int n) {
  std::vector<float> h(n);
  CK(hipMemcpy(h.data(), dA, n * sizeof(float), hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < n; ++i) bad += h[i] != 1.f;
  return bad;
}

// n: A's words; nb: B's words; eager: eager memsets between replays; other_stream: B's memsets on
// a second stream (else the replay stream)
static void run_case(int n, int nb, int eager, bool other_stream, int rounds) {
  float *A, *B;
  CK(hipMalloc(&A, n * sizeof(float)));
  CK(hipMalloc(&B, nb * sizeof(float)));
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  CK(hipMemsetAsync(A, 0, n * sizeof(float), s));
  hipLaunchKernelGGL(add_one, dim3((n + 255) / 256), dim3(256), 0, s, A, n);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  std::printf("n=%d nb=%d eager=%d %s:", n, nb, eager, other_stream ? "other-stream" : "same-stream");
  for (int r = 0; r < rounds; ++r) {
    hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, s, A, n, 12345.f);  // sentinel
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    std::printf(" r%d=%d", r, count_bad(A, n));
    hipStream_t es = other_stream ? s2 : s;
    for (int k = 0; k < eager; ++k) {
      CK(hipMemsetAsync(B, 0, nb * sizeof(float), es));
      hipLaunchKernelGGL(add_one, dim3((nb + 255) / 256), dim3(256), 0, es, B, nb);
    }
    CK(hipStreamSynchronize(es));
  }
  std::printf("\n");
  std::fflush(stdout);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(s));
  CK(hipStreamDestroy(s2));
  CK(hipFree(A));
  CK(hipFree(B));
}

int main() {
  const int sizes[][2] = {{1000, 1000}, {1000, 4096}, {4096, 1000}, {1 << 20, 1 << 20}, {1 << 20, 1000}, {250, 250}};
  for (auto& sz : sizes)
    for (int eager : {0, 4})
      for (bool other : {false, true}) run_case(sz[0], sz[1], eager, other, 4);
  return 0;
}
