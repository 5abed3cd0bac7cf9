// Memset nodes of a captured hipGraph rewritten as kernel nodes (utils/graphs.py GraphedStep).
//
// A ResNet-50 step captured with MIOpen's exhaustive-find solvers holds hipMemsetAsync nodes
// (the atomic weight-gradient solvers zero their outputs first). Replays of such graphs diverged
// (profiles/r4_graph_memset.md): the deterministic-solver build (no memsets) replays bit-exactly,
// and round 3 saw a captured memset leave 250 of 1,000 floats unzeroed. A kernel node doing the
// same fill takes the runtime's memset-node path out of the replay. The graph is edited before
// instantiation (torch.cuda.CUDAGraph(keep_graph=True)): every memset node is replaced by a
// kernel node with the same dependencies and dependents.
#include <vector>

#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

// value: the memset's element value (1, 2 or 4 bytes wide); rows of `width` elements, `pitch` bytes apart
__global__ void __launch_bounds__(256) graph_fill_kernel(uint8_t* __restrict__ dst, size_t pitch, size_t width,
                                                         size_t height, int esize, uint32_t value) {
  const size_t total = width * height;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const size_t r = e / width, c = e - r * width;
    uint8_t* p = dst + r * pitch + c * esize;
    if (esize == 4) *reinterpret_cast<uint32_t*>(p) = value;
    else if (esize == 2) *reinterpret_cast<uint16_t*>(p) = (uint16_t)value;
    else *p = (uint8_t)value;
  }
}

}  // namespace

int graph_node_census(void* graph, int* counts, int ncounts) {
  hipGraph_t g = static_cast<hipGraph_t>(graph);
  size_t n = 0;
  if (hipGraphGetNodes(g, nullptr, &n) != hipSuccess) return -1;
  std::vector<hipGraphNode_t> nodes(n);
  if (n && hipGraphGetNodes(g, nodes.data(), &n) != hipSuccess) return -1;
  for (int i = 0; i < ncounts; ++i) counts[i] = 0;
  for (auto nd : nodes) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nd, &t) != hipSuccess) return -1;
    if ((int)t >= 0 && (int)t < ncounts) ++counts[(int)t];
  }
  return (int)n;
}

int graph_replace_memsets(void* graph) {
  hipGraph_t g = static_cast<hipGraph_t>(graph);
  size_t n = 0;
  if (hipGraphGetNodes(g, nullptr, &n) != hipSuccess) return -1;
  std::vector<hipGraphNode_t> nodes(n);
  if (n && hipGraphGetNodes(g, nodes.data(), &n) != hipSuccess) return -1;
  int replaced = 0;
  for (auto nd : nodes) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nd, &t) != hipSuccess) return -1;
    if (t != hipGraphNodeTypeMemset) continue;
    hipMemsetParams mp{};
    if (hipGraphMemsetNodeGetParams(nd, &mp) != hipSuccess) return -1;
    if (mp.elementSize != 1 && mp.elementSize != 2 && mp.elementSize != 4) return -1;
    size_t nd_in = 0, nd_out = 0;
    if (hipGraphNodeGetDependencies(nd, nullptr, &nd_in) != hipSuccess) return -1;
    if (hipGraphNodeGetDependentNodes(nd, nullptr, &nd_out) != hipSuccess) return -1;
    std::vector<hipGraphNode_t> ins(nd_in), outs(nd_out);
    if (nd_in && hipGraphNodeGetDependencies(nd, ins.data(), &nd_in) != hipSuccess) return -1;
    if (nd_out && hipGraphNodeGetDependentNodes(nd, outs.data(), &nd_out) != hipSuccess) return -1;
    uint8_t* dst = static_cast<uint8_t*>(mp.dst);
    size_t pitch = mp.pitch ? mp.pitch : mp.width * mp.elementSize;
    size_t width = mp.width, height = mp.height ? mp.height : 1;
    int esize = (int)mp.elementSize;
    uint32_t value = mp.value;
    const size_t total = width * height;
    const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>((total + 255) / 256, 2048));
    void* args[] = {&dst, &pitch, &width, &height, &esize, &value};
    hipKernelNodeParams kp{};
    kp.func = reinterpret_cast<void*>(&graph_fill_kernel);
    kp.gridDim = dim3(blocks);
    kp.blockDim = dim3(256);
    kp.sharedMemBytes = 0;
    kp.kernelParams = args;
    kp.extra = nullptr;
    hipGraphNode_t kn;
    if (hipGraphAddKernelNode(&kn, g, ins.empty() ? nullptr : ins.data(), ins.size(), &kp) != hipSuccess) return -1;
    for (auto o : outs)
      if (hipGraphAddDependencies(g, &kn, &o, 1) != hipSuccess) return -1;
    if (hipGraphDestroyNode(nd) != hipSuccess) return -1;
    ++replaced;
  }
  return replaced;
}

// Parameters of every memset node (graph order): dst, value, elementSize, width, height, pitch.
int graph_memset_params(void* graph, std::vector<std::vector<int64_t>>* out) {
  hipGraph_t g = static_cast<hipGraph_t>(graph);
  size_t n = 0;
  if (hipGraphGetNodes(g, nullptr, &n) != hipSuccess) return -1;
  std::vector<hipGraphNode_t> nodes(n);
  if (n && hipGraphGetNodes(g, nodes.data(), &n) != hipSuccess) return -1;
  out->clear();
  for (auto nd : nodes) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nd, &t) != hipSuccess) return -1;
    if (t != hipGraphNodeTypeMemset) continue;
    hipMemsetParams mp{};
    if (hipGraphMemsetNodeGetParams(nd, &mp) != hipSuccess) return -1;
    out->push_back({(int64_t)reinterpret_cast<uintptr_t>(mp.dst), (int64_t)mp.value, (int64_t)mp.elementSize,
                    (int64_t)mp.width, (int64_t)mp.height, (int64_t)mp.pitch});
  }
  return (int)out->size();
}

// One memset node with the given parameters in a fresh graph, instantiated and launched
// `reps` times on stream s (synchronised): the runtime's memset-node path in isolation.
hipError_t graph_memset_run(void* dst, uint32_t value, int esize, size_t width, size_t height, size_t pitch,
                            int reps, hipStream_t s) {
  hipGraph_t g = nullptr;
  PTDT_HIP_CHECK(hipGraphCreate(&g, 0));
  hipMemsetParams mp{};
  mp.dst = dst;
  mp.value = value;
  mp.elementSize = (unsigned)esize;
  mp.width = width;
  mp.height = height;
  mp.pitch = pitch;
  hipGraphNode_t nd;
  hipError_t e = hipGraphAddMemsetNode(&nd, g, nullptr, 0, &mp);
  hipGraphExec_t ex = nullptr;
  if (e == hipSuccess) e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  for (int r = 0; r < reps && e == hipSuccess; ++r) e = hipGraphLaunch(ex, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (ex) hipGraphExecDestroy(ex);
  hipGraphDestroy(g);
  return e;
}

}  // namespace ptdt
