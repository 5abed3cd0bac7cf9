// Throughput bf16 GEMM for gfx950: LDS-DMA staging, double-buffered 64-deep
// K-tiles, XCD-aware tile order, Linear-layer epilogue fused, optional split-K.
//
//   C[M,N] = alpha * A[M,K] . Bt[N,K]^T (+ beta*C) (+ bias[N]) (ReLU)
//
// Both operands are K-contiguous (row-major A, and B given as its transpose
// Bt[N,K] -- exactly nn.Linear's weight layout, so y = x W^T needs no copy).
// This is the throughput path of ops/linear.py; the strided 64x64 kernel in
// gemm.hip keeps the odd layouts and fusions (ReLU mask on A, bias-grad row
// sums) for the small and latency-bound shapes.
//
// Two block tiles (one template, host picks by how many tiles fill 256 CUs):
//   T256: 256x256, 512 threads = 8 waves as 2 (M) x 4 (N), each wave a 128x64
//         sub-tile = 8x4 v_mfma_f32_16x16x32_bf16 accumulators; 128 KiB LDS,
//         one workgroup per CU; ping-pong wave pairs (SCHED 1, below).
//   T128: 128x128, 256 threads = 4 waves as 2 x 2, each wave 64x64 = 4x4
//         accumulators; 64 KiB LDS so two workgroups share a CU and overlap
//         each other's LDS reads with MFMAs. For mid-size shapes where 256x256
//         tiles leave most of the 256 CUs idle (2048^2 has 64 such tiles).
//   split-K (gridDim.y > 1): each workgroup reduces a contiguous range of
//         K-tiles and fp32-atomically adds into a pre-zeroed f32 C (bias from
//         slice 0); for small-MN / long-K shapes (ResNet fc 120x1000x2048).
//
// Common structure (cdna_hip_programming.md §5, "glds, 2 LDS buffers, BK=64"):
//   * global -> LDS with global_load_lds_dwordx4 (16 B per lane, no VGPR
//     round trip): each wave-instruction fills 1 KiB of LDS linearly, so the
//     bank swizzle is applied to the per-lane SOURCE address and undone on the
//     ds_read side (same involution on both sides).
//   * swizzle: a tile is rows x 8 chunks of 16 B; chunk c of row r lives in
//     slot c ^ ((r >> 1) & 7). The 16 lanes of a ds_read_b128 (16 consecutive
//     rows, same logical chunk) hit 16 distinct 16-B slots: conflict-free.
//   * pipeline: tile k+1 is in flight (its LDS-DMA counted on vmcnt) while tile
//     k is multiplied; a counted `s_waitcnt vmcnt(N)` + raw s_barrier retires
//     exactly tile k (never vmcnt(0) in the steady state, never __syncthreads,
//     whose fence would drain the prefetch), and a second barrier after the
//     fragment reads frees the buffer for tile k+2.
//   * edges: rows/cols past M/N read a clamped (valid) row and are not stored;
//     K must be a multiple of 64 (host checks), bases 16-B aligned.
#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

constexpr int BK = 64;

template <int BM_, int BN_, int WM_, int WN_>
struct Tile {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
  static constexpr int NT = WM * WN * 64;
  static constexpr int TA = BM * BK * 2, TB = BN * BK * 2;  // operand tile bytes
  static constexpr int BUF = TA + TB;
  static constexpr int LDS = 2 * BUF;                        // double buffered
  static constexpr int FI = BM / WM / 16, FJ = BN / WN / 16;  // MFMA tiles per wave
  static constexpr int VM = TA / (NT * 16) + TB / (NT * 16);  // LDS-DMAs per thread per K-tile
  static_assert(TA % (NT * 16) == 0 && TB % (NT * 16) == 0, "tile not a whole number of DMA rounds");
};
using T256 = Tile<256, 256, 2, 4>;
using T128 = Tile<128, 128, 2, 2>;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N == 8, "add the literal for this DMA count");
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
}

// Issue the LDS-DMA of one ROWS x 64 operand tile (rows row0.., k0..k0+63) with THREADS threads.
template <int ROWS, int THREADS>
__device__ __forceinline__ void stage_tile(const uint16_t* __restrict__ src, int64_t ld, int row0, int nrows,
                                           int k0, uint8_t* lds_tile, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < ROWS * BK * 2 / (THREADS * 16); ++i) {
    const int p = i * THREADS + wid * 64 + lane;  // linear 16-B chunk index in the tile image
    const int r = p >> 3, slot = p & 7;
    const int c = slot ^ ((r >> 1) & 7);      // logical k-chunk stored in this slot
    const int gr = min(row0 + r, nrows - 1);  // clamp: edge rows are computed, never stored
    const uint16_t* g = src + (int64_t)gr * ld + k0 + c * 8;
    // wave-uniform LDS base; the hardware adds lane * 16
    uint8_t* dst = lds_tile + (i * THREADS + wid * 64) * 16;
    __builtin_amdgcn_global_load_lds((gbl_void*)g, (lds_void*)dst, 16, 0, 0);
  }
}

template <class T>
__device__ __forceinline__ void stage(const uint16_t* A, int64_t lda, int m0, int M, const uint16_t* Bt,
                                      int64_t ldb, int n0, int N, int k0, uint8_t* buf, int wid, int lane) {
  stage_tile<T::BM, T::NT>(A, lda, m0, M, k0, buf, wid, lane);
  stage_tile<T::BN, T::NT>(Bt, ldb, n0, N, k0, buf + T::TA, wid, lane);
}

__device__ __forceinline__ bf16x8_t read_frag(const uint8_t* lds_tile, int row, int c) {
  const int slot = c ^ ((row >> 1) & 7);
  return *reinterpret_cast<const bf16x8_t*>(lds_tile + row * (BK * 2) + slot * 16);
}

// Fragment reads of one 64-deep K-tile for a wave's sub-tile.
template <class T>
struct Frags {
  bf16x8_t a[2][T::FI], b[2][T::FJ];
};

template <class T>
__device__ __forceinline__ void read_tile(Frags<T>& f, const uint8_t* at, const uint8_t* bt, int wr, int wc, int fr,
                                          int fq) {
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
    for (int j = 0; j < T::FJ; ++j) f.b[kb][j] = read_frag(bt, wc * (T::FJ * 16) + j * 16 + fr, kb * 4 + fq);
#pragma unroll
    for (int i = 0; i < T::FI; ++i) f.a[kb][i] = read_frag(at, wr * (T::FI * 16) + i * 16 + fr, kb * 4 + fq);
  }
}

template <class T>
__device__ __forceinline__ void mfma_tile(f32x4_t (&acc)[T::FI][T::FJ], const Frags<T>& f) {
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int i = 0; i < T::FI; ++i)
#pragma unroll
      for (int j = 0; j < T::FJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[kb][i], f.b[kb][j], acc[i][j], 0, 0, 0);
}

// OUT: 0 bf16 store, 1 f32 store, 2 f32 atomic add (split-K slices).
// SCHED 0: every wave reads then multiplies each K-tile (two barriers per tile,
//          tile k+1's DMA in flight meanwhile).
// SCHED 1: ping-pong (T256 only). The two waves sharing a SIMD (wave w and w+4:
//          the M-halves wr = 0 / 1) run half a tile apart: while one multiplies
//          K-tile t from registers, its partner reads K-tile t's fragments from
//          LDS, so the SIMD's matrix pipe always has one wave feeding it. Slots
//          are separated by workgroup barriers; wr=1 waves start one slot late.
//          Tile t+1's DMA is issued at the start of slot 2t and retired
//          (vmcnt(0)) before the barrier closing slot 2t+1: its buffer's previous
//          tile (t-1) was last read in slot 2t-1, and its first reader starts in
//          slot 2t+2.
template <class T, int OUT, int SCHED>
__global__ void __launch_bounds__(T::NT) gemm_bf16_lds_kernel(BigGemmArgs g, int tm, int tn, int kt_per) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tile = xcd_remap(blockIdx.x, tm * tn);
  const int bm = tile / tn, bn = tile % tn;
  const int m0 = bm * T::BM, n0 = bn * T::BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / T::WN, wc = wid % T::WN;
  const uint16_t* A = static_cast<const uint16_t*>(g.A);
  const uint16_t* Bt = static_cast<const uint16_t*>(g.Bt);
  const int nk_all = g.K / BK;
  const int kt_begin = blockIdx.y * kt_per;
  const int nk = min(nk_all, kt_begin + kt_per) - kt_begin;  // >= 1 (host sizes the split)
  const int kbase = kt_begin * BK;
  const int fr = lane & 15, fq = lane >> 4;

  f32x4_t acc[T::FI][T::FJ];
#pragma unroll
  for (int i = 0; i < T::FI; ++i)
#pragma unroll
    for (int j = 0; j < T::FJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  stage<T>(A, g.lda, m0, g.M, Bt, g.ldb, n0, g.N, kbase, smem, wid, lane);

  if constexpr (SCHED == 0) {
    for (int kt = 0; kt < nk; ++kt) {
      uint8_t* cur = smem + (kt & 1) * T::BUF;
      if (kt + 1 < nk) {
        stage<T>(A, g.lda, m0, g.M, Bt, g.ldb, n0, g.N, kbase + (kt + 1) * BK, smem + ((kt + 1) & 1) * T::BUF,
                 wid, lane);
        wait_vmcnt<T::VM>();  // tile kt landed, kt+1 still in flight
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();  // every wave's DMA of tile kt is visible
      __builtin_amdgcn_sched_barrier(0);
      Frags<T> f;
      read_tile<T>(f, cur, cur + T::TA, wr, wc, fr, fq);
      mfma_tile<T>(acc, f);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();  // buffer kt&1 free for tile kt+2
    }
  } else {
    static_assert(T::WM == 2 && T::NT == 512, "ping-pong pairs waves w and w+4 on one SIMD");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // tile 0 visible
    __builtin_amdgcn_sched_barrier(0);
    Frags<T> f;
    // one loop per role (same barrier count): the register allocator then
    // sees the fragments live only between their read and their MFMAs
    if (wr == 0) {  // leader: slot 2kt reads tile kt, slot 2kt+1 multiplies it
      for (int kt = 0; kt < nk; ++kt) {
        const uint8_t* cur = smem + (kt & 1) * T::BUF;
        if (kt + 1 < nk)
          stage<T>(A, g.lda, m0, g.M, Bt, g.ldb, n0, g.N, kbase + (kt + 1) * BK, smem + ((kt + 1) & 1) * T::BUF,
                   wid, lane);
        read_tile<T>(f, cur, cur + T::TA, wr, wc, fr, fq);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        mfma_tile<T>(acc, f);
        __builtin_amdgcn_s_setprio(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile kt+1 landed (own DMA)
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {  // follower: slot 2kt multiplies tile kt-1, slot 2kt+1 reads tile kt
      for (int kt = 0; kt < nk; ++kt) {
        const uint8_t* cur = smem + (kt & 1) * T::BUF;
        if (kt + 1 < nk)
          stage<T>(A, g.lda, m0, g.M, Bt, g.ldb, n0, g.N, kbase + (kt + 1) * BK, smem + ((kt + 1) & 1) * T::BUF,
                   wid, lane);
        if (kt > 0) {
          __builtin_amdgcn_s_setprio(1);
          mfma_tile<T>(acc, f);
          __builtin_amdgcn_s_setprio(0);
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        read_tile<T>(f, cur, cur + T::TA, wr, wc, fr, fq);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
      mfma_tile<T>(acc, f);
    }
  }

  // epilogue: acc[i][j][r] = C[m0 + wr*FI*16 + i*16 + 4*fq + r][n0 + wc*FJ*16 + j*16 + fr]
  const bool add_bias = g.bias != nullptr && blockIdx.y == 0;
#pragma unroll
  for (int j = 0; j < T::FJ; ++j) {
    const int n = n0 + wc * (T::FJ * 16) + j * 16 + fr;
    if (n >= g.N) continue;
    float bias = 0.f;
    if (add_bias)
      bias = g.bias_dtype == kF32 ? static_cast<const float*>(g.bias)[n]
                                  : bf16_to_f32(static_cast<const uint16_t*>(g.bias)[n]);
#pragma unroll
    for (int i = 0; i < T::FI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * (T::FI * 16) + i * 16 + 4 * fq + r;
        if (m >= g.M) continue;
        const int64_t off = (int64_t)m * g.ldc + n;
        float v = g.alpha * acc[i][j][r];
        if constexpr (OUT == 2) {
          atomicAdd(static_cast<float*>(g.C) + off, v + bias);
        } else if constexpr (OUT == 1) {
          float* c = static_cast<float*>(g.C);
          if (g.beta != 0.f) v += g.beta * c[off];
          v += bias;
          c[off] = g.relu ? fmaxf(v, 0.f) : v;
        } else {
          uint16_t* c = static_cast<uint16_t*>(g.C);
          if (g.beta != 0.f) v += g.beta * bf16_to_f32(c[off]);
          v += bias;
          c[off] = f32_to_bf16(g.relu ? fmaxf(v, 0.f) : v);
        }
      }
  }
}

template <class T, int OUT, int SCHED>
hipError_t launch(const BigGemmArgs& g, int split, hipStream_t s) {
  const void* fn = reinterpret_cast<const void*>(&gemm_bf16_lds_kernel<T, OUT, SCHED>);
  static bool attr_set = false;  // one flag per instantiation
  if (!attr_set) {
    PTDT_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, T::LDS));
    attr_set = true;
  }
  const int tm = (g.M + T::BM - 1) / T::BM, tn = (g.N + T::BN - 1) / T::BN;
  const int nk = g.K / BK;
  const int kt_per = (nk + split - 1) / split;
  split = (nk + kt_per - 1) / kt_per;  // no empty slices
  hipLaunchKernelGGL((gemm_bf16_lds_kernel<T, OUT, SCHED>), dim3(tm * tn, split), dim3(T::NT), T::LDS, s, g, tm,
                     tn, kt_per);
  return hipGetLastError();
}

template <class T, int SCHED>
hipError_t launch_out(const BigGemmArgs& g, int split, hipStream_t s) {
  if (split > 1) return launch<T, 2, SCHED>(g, split, s);
  return g.out_dtype == kF32 ? launch<T, 1, SCHED>(g, 1, s) : launch<T, 0, SCHED>(g, 1, s);
}

}  // namespace

bool gemm_bf16_big_supported(int M, int N, int K, int64_t lda, int64_t ldb, const void* A, const void* Bt) {
  return M > 0 && N > 0 && K >= BK && K % BK == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         (reinterpret_cast<uintptr_t>(A) & 15) == 0 && (reinterpret_cast<uintptr_t>(Bt) & 15) == 0;
}

hipError_t gemm_bf16_big(const BigGemmArgs& g, hipStream_t s) {
  if (!gemm_bf16_big_supported(g.M, g.N, g.K, g.lda, g.ldb, g.A, g.Bt)) return hipErrorInvalidValue;
  const int split = g.split_k > 1 ? g.split_k : 1;
  // split-K slices accumulate with fp32 atomics: f32 C (pre-zeroed by the caller), no ReLU/beta
  if (split > 1 && (g.out_dtype != kF32 || g.relu || g.beta != 0.f)) return hipErrorInvalidValue;
  if (g.tile == 128) {
    if (g.sched != 0 && g.sched != 1) return hipErrorInvalidValue;
    return launch_out<T128, 0>(g, split, s);  // 4 waves, one per SIMD: no ping-pong partner
  }
  if (g.tile != 256) return hipErrorInvalidValue;
  if (g.sched == 0) return launch_out<T256, 0>(g, split, s);
  if (g.sched == 1) return launch_out<T256, 1>(g, split, s);
  return hipErrorInvalidValue;
}

}  // namespace ptdt
