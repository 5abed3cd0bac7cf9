// LDS-tiled MFMA GEMM for gfx950 with the Linear-layer epilogues fused.
//
//   C[M,N] = alpha * A[M,K] . B[K,N] (+ beta*C) (+ bias[N]) (ReLU)
//
// A and B are addressed through (row, col) strides, so the three products of a
// Linear layer -- y = x W^T (NT), dx = dy W (NN), dW = dy^T x (TN) -- run on
// the same kernel without transposed copies. Optional fusions:
//   * ReLU-backward mask on the A operand (dy * (y > 0)) applied while staging,
//   * row sums of the (masked) A operand -> bias gradients in the dW launch,
//   * bias + ReLU epilogue for the forward,
//   * split-K over blockIdx.y with fp32 atomics for long-K / tiny-MN shapes
//     (the reference's Linear(10000,10) stage, NB03:449, K=10000).
//
// Two instruction paths (cdna_hip_programming.md §3):
//   bf16: v_mfma_f32_16x16x32_bf16, 64x64x32 block tile, 4 waves each owning
//         a 32x32 sub-tile = 2x2 MFMA tiles; fragments read with 16-B LDS reads
//         from k-contiguous images padded to 80-B rows (conflict-free).
//   f32 : v_mfma_f32_32x32x2_f32 (exact fp32 FMA chain, no xf32 on CDNA4),
//         64x64x16 block tile, one 32x32 accumulator per wave, odd LDS stride.
// Workgroups are remapped XCD-aware so neighbouring tiles share an L2.
#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

constexpr int kThreads = 256;
constexpr int BM = 64, BN = 64;

template <typename T>
__device__ __forceinline__ float ld(const void* p, int64_t i) {
  return Cvt<T>::load(static_cast<const T*>(p), i);
}

__device__ __forceinline__ float load_bias(const GemmArgs& g, int n) {
  return g.bias_dtype == kF32 ? static_cast<const float*>(g.bias)[n]
                              : bf16_to_f32(static_cast<const uint16_t*>(g.bias)[n]);
}

__device__ __forceinline__ void store_out(const GemmArgs& g, int m, int n, float v, bool atomic) {
  const int64_t off = (int64_t)m * g.scm + (int64_t)n * g.scn;
  if (g.out_dtype == kF32) {
    float* c = static_cast<float*>(g.C);
    if (atomic) {
      atomicAdd(c + off, v);
      return;
    }
    if (g.beta != 0.f) v += g.beta * c[off];
    c[off] = v;
  } else {
    uint16_t* c = static_cast<uint16_t*>(g.C);
    if (g.beta != 0.f) v += g.beta * bf16_to_f32(c[off]);
    c[off] = f32_to_bf16(v);
  }
}

// Stage a BROWS x BK tile of A (rows = m) or of B^T (rows = n) into a
// k-contiguous LDS image with row stride LDK. `rs`, `cs`: source strides of
// (row, k). Coalesced for both k-contiguous and row-contiguous sources.
template <typename TIn, typename TL, int BROWS, int BK, int LDK>
__device__ __forceinline__ void stage(TL* lds, const void* src, int64_t rs, int64_t ks, int row0,
                                      int nrows, int k0, int K, const void* mask, int64_t mrs,
                                      int64_t mks) {
  constexpr int kElems = BROWS * BK;
  const int tid = threadIdx.x;
  const bool kcontig = (ks == 1);
#pragma unroll
  for (int j = 0; j < kElems / kThreads; ++j) {
    const int e = j * kThreads + tid;
    int r, k;
    if (kcontig) {
      r = e / BK;
      k = e % BK;
    } else {
      r = e % BROWS;
      k = e / BROWS;
    }
    const int gr = row0 + r, gk = k0 + k;
    float v = 0.f;
    if (gr < nrows && gk < K) {
      v = ld<TIn>(src, (int64_t)gr * rs + (int64_t)gk * ks);
      if (mask != nullptr && ld<TIn>(mask, (int64_t)gr * mrs + (int64_t)gk * mks) <= 0.f) v = 0.f;
    }
    if constexpr (sizeof(TL) == 2)
      lds[r * LDK + k] = f32_to_bf16(v);
    else
      lds[r * LDK + k] = v;
  }
}

// ------------------------------------------------------------------ bf16 path
template <typename TIn>
__global__ void __launch_bounds__(kThreads) gemm_bf16_kernel(GemmArgs g, int tm, int tn, int kt_per) {
  constexpr int BK = 32, LDK = BK + 8;
  __shared__ __attribute__((aligned(16))) uint16_t As[BM * LDK];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[BN * LDK];
  const int tile = xcd_remap(blockIdx.x, tm * tn);
  const int bm = tile / tn, bn = tile % tn;
  const int m0 = bm * BM, n0 = bn * BN;
  const int ktiles = (g.K + BK - 1) / BK;
  const int kt0 = blockIdx.y * kt_per, kt1 = min(ktiles, kt0 + kt_per);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const bool do_rowsum = g.colsum_out != nullptr && bn == 0;
  float rsum = 0.f;

  f32x4_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int kt = kt0; kt < kt1; ++kt) {
    const int k0 = kt * BK;
    stage<TIn, uint16_t, BM, BK, LDK>(As, g.A, g.sam, g.sak, m0, g.M, k0, g.K, g.amask, g.smm, g.smk);
    stage<TIn, uint16_t, BN, BK, LDK>(Bs, g.B, g.sbn, g.sbk, n0, g.N, k0, g.K, nullptr, 0, 0);
    __syncthreads();
    if (do_rowsum && threadIdx.x < BM) {
      for (int k = 0; k < BK; ++k) rsum += bf16_to_f32(As[threadIdx.x * LDK + k]);
    }
    bf16x8_t af[2], bfr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = wr * 32 + i * 16 + (lane & 15);
      af[i] = *reinterpret_cast<const bf16x8_t*>(&As[row * LDK + 8 * (lane >> 4)]);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = wc * 32 + j * 16 + (lane & 15);
      bfr[j] = *reinterpret_cast<const bf16x8_t*>(&Bs[col * LDK + 8 * (lane >> 4)]);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    __syncthreads();
  }

  if (do_rowsum && threadIdx.x < BM && m0 + (int)threadIdx.x < g.M)
    atomicAdd(g.colsum_out + m0 + threadIdx.x, rsum);

  const bool atomic = gridDim.y > 1;
  const bool add_bias = g.bias != nullptr && (!atomic || blockIdx.y == 0);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * 32 + i * 16 + (lane >> 4) * 4 + r;
        const int n = n0 + wc * 32 + j * 16 + (lane & 15);
        if (m < g.M && n < g.N) {
          float v = g.alpha * acc[i][j][r];
          if (add_bias) v += load_bias(g, n);
          if (g.relu) v = fmaxf(v, 0.f);
          store_out(g, m, n, v, atomic);
        }
      }
}

// ------------------------------------------------------------------- f32 path
__global__ void __launch_bounds__(kThreads) gemm_f32_kernel(GemmArgs g, int tm, int tn, int kt_per) {
  constexpr int BK = 16, LDK = BK + 1;
  __shared__ float As[BM * LDK];
  __shared__ float Bs[BN * LDK];
  const int tile = xcd_remap(blockIdx.x, tm * tn);
  const int bm = tile / tn, bn = tile % tn;
  const int m0 = bm * BM, n0 = bn * BN;
  const int ktiles = (g.K + BK - 1) / BK;
  const int kt0 = blockIdx.y * kt_per, kt1 = min(ktiles, kt0 + kt_per);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const bool do_rowsum = g.colsum_out != nullptr && bn == 0;
  float rsum = 0.f;
  f32x16_t acc = {};

  for (int kt = kt0; kt < kt1; ++kt) {
    const int k0 = kt * BK;
    stage<float, float, BM, BK, LDK>(As, g.A, g.sam, g.sak, m0, g.M, k0, g.K, g.amask, g.smm, g.smk);
    stage<float, float, BN, BK, LDK>(Bs, g.B, g.sbn, g.sbk, n0, g.N, k0, g.K, nullptr, 0, 0);
    __syncthreads();
    if (do_rowsum && threadIdx.x < BM) {
      for (int k = 0; k < BK; ++k) rsum += As[threadIdx.x * LDK + k];
    }
    const float* ar = &As[(wr * 32 + (lane & 31)) * LDK + (lane >> 5)];
    const float* br = &Bs[(wc * 32 + (lane & 31)) * LDK + (lane >> 5)];
#pragma unroll
    for (int s = 0; s < BK / 2; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[2 * s], br[2 * s], acc, 0, 0, 0);
    __syncthreads();
  }

  if (do_rowsum && threadIdx.x < BM && m0 + (int)threadIdx.x < g.M)
    atomicAdd(g.colsum_out + m0 + threadIdx.x, rsum);

  const bool atomic = gridDim.y > 1;
  const bool add_bias = g.bias != nullptr && (!atomic || blockIdx.y == 0);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    const int n = n0 + wc * 32 + (lane & 31);
    if (m < g.M && n < g.N) {
      float v = g.alpha * acc[r];
      if (add_bias) v += load_bias(g, n);
      if (g.relu) v = fmaxf(v, 0.f);
      store_out(g, m, n, v, atomic);
    }
  }
}

}  // namespace

hipError_t gemm(const GemmArgs& g, hipStream_t s) {
  if (g.M <= 0 || g.N <= 0) return hipSuccess;
  if (g.K < 0) return hipErrorInvalidValue;
  const int tm = (g.M + BM - 1) / BM, tn = (g.N + BN - 1) / BN;
  const int bk = g.in_dtype == kF32 ? 16 : 32;
  const int ktiles = (g.K + bk - 1) / bk;
  int split = g.split_k > 1 ? g.split_k : 1;
  if (split > ktiles) split = ktiles > 0 ? ktiles : 1;
  if (split > 1 && (g.out_dtype != kF32 || g.relu || g.beta != 0.f)) return hipErrorInvalidValue;
  const int kt_per = ktiles > 0 ? (ktiles + split - 1) / split : 0;
  split = kt_per > 0 ? (ktiles + kt_per - 1) / kt_per : 1;
  GemmArgs a = g;
  if (split > 1) a.split_k = split;
  dim3 grid(tm * tn, split);
  if (g.in_dtype == kF32) {
    hipLaunchKernelGGL(gemm_f32_kernel, grid, dim3(kThreads), 0, s, a, tm, tn, kt_per);
  } else {
    hipLaunchKernelGGL(gemm_bf16_kernel<uint16_t>, grid, dim3(kThreads), 0, s, a, tm, tn, kt_per);
  }
  return hipGetLastError();
}

}  // namespace ptdt
