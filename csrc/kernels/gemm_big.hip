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

// Epilogue of a wave's FI x FJ accumulator tiles:
// acc[i][j][r] = C[m0 + wr*FI*16 + i*16 + 4*fq + r][n0 + wc*FJ*16 + j*16 + fr]
template <int FI, int FJ, int OUT>
__device__ __forceinline__ void store_tile(const BigGemmArgs& g, const f32x4_t (&acc)[FI][FJ], int m0, int n0, int wr,
                                           int wc, int fr, int fq) {
  const bool add_bias = g.bias != nullptr && blockIdx.y == 0;
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    const int n = n0 + wc * (FJ * 16) + j * 16 + fr;
    if (n >= g.N) continue;
    float bias = 0.f;
    if (add_bias)
      bias = g.bias_dtype == kF32 ? static_cast<const float*>(g.bias)[n]
                                  : bf16_to_f32(static_cast<const uint16_t*>(g.bias)[n]);
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * (FI * 16) + i * 16 + 4 * fq + r;
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

// Coalesced epilogue (OUT 0 / 1): the accumulators of 64-row bands go through LDS (fp32, row
// stride FJ*16 + 4 floats: the four lane groups of a write land on distinct banks), then each lane
// finishes 8 consecutive columns of a row -- alpha, beta*C, bias, ReLU -- and writes them with one
// 16-B (bf16) or two 16-B (f32) stores instead of 8 scattered 2/4-B stores per 8 outputs.
// `scratch` is this wave's LDS region of epi_floats<FJ>() floats; the caller has made every wave
// finish its operand reads (barrier) before the first band is written.
template <int FJ>
constexpr int epi_ld() { return FJ * 16 + 4; }
template <int FJ>
constexpr int epi_floats() { return 64 * epi_ld<FJ>(); }

template <int FI, int FJ, int OUT>
__device__ __forceinline__ void store_tile_lds(const BigGemmArgs& g, const f32x4_t (&acc)[FI][FJ], int m0, int n0,
                                               int wr, int wc, int fr, int fq, float* scratch) {
  static_assert(OUT == 0 || OUT == 1, "split-K slices use the atomic epilogue");
  static_assert(FI % 4 == 0, "64-row bands");
  constexpr int LD = epi_ld<FJ>(), W = FJ * 16, CPR = W / 8;  // columns per wave row, 8-column chunks per row
  const int lane = fr + 16 * fq;
  const bool add_bias = g.bias != nullptr;
  const int ncol0 = n0 + wc * W;
  const bool vec = (g.ldc % 8 == 0) && ((reinterpret_cast<uintptr_t>(g.C) & 15) == 0);
#pragma unroll
  for (int band = 0; band < FI / 4; ++band) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) scratch[(i * 16 + 4 * fq + r) * LD + j * 16 + fr] = acc[band * 4 + i][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const int mrow0 = m0 + wr * (FI * 16) + band * 64;
#pragma unroll
    for (int it = 0; it < 64 * CPR / 64; ++it) {
      const int e = it * 64 + lane;  // (row, chunk) of this lane
      const int row = e / CPR, ch = e % CPR;
      const int m = mrow0 + row, n = ncol0 + ch * 8;
      const float4 lo = *reinterpret_cast<const float4*>(scratch + row * LD + ch * 8);
      const float4 hi = *reinterpret_cast<const float4*>(scratch + row * LD + ch * 8 + 4);
      float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      if (m >= g.M || n >= g.N) continue;
      const bool full = vec && n + 8 <= g.N;
      const int64_t off = (int64_t)m * g.ldc + n;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int nn = n + q;
        float x = g.alpha * v[q];
        if (nn < g.N) {
          if (g.beta != 0.f)
            x += g.beta * (OUT == 1 ? static_cast<const float*>(g.C)[off + q]
                                    : bf16_to_f32(static_cast<const uint16_t*>(g.C)[off + q]));
          if (add_bias)
            x += g.bias_dtype == kF32 ? static_cast<const float*>(g.bias)[nn]
                                      : bf16_to_f32(static_cast<const uint16_t*>(g.bias)[nn]);
        }
        v[q] = g.relu ? fmaxf(x, 0.f) : x;
      }
      if constexpr (OUT == 1) {
        float* c = static_cast<float*>(g.C) + off;
        if (full) {
          *reinterpret_cast<float4*>(c) = make_float4(v[0], v[1], v[2], v[3]);
          *reinterpret_cast<float4*>(c + 4) = make_float4(v[4], v[5], v[6], v[7]);
        } else {
          for (int q = 0; q < 8 && n + q < g.N; ++q) c[q] = v[q];
        }
      } else {
        uint16_t* c = static_cast<uint16_t*>(g.C) + off;
        if (full) {
          uint4 u;
          u.x = (uint32_t)f32_to_bf16(v[0]) | ((uint32_t)f32_to_bf16(v[1]) << 16);
          u.y = (uint32_t)f32_to_bf16(v[2]) | ((uint32_t)f32_to_bf16(v[3]) << 16);
          u.z = (uint32_t)f32_to_bf16(v[4]) | ((uint32_t)f32_to_bf16(v[5]) << 16);
          u.w = (uint32_t)f32_to_bf16(v[6]) | ((uint32_t)f32_to_bf16(v[7]) << 16);
          *reinterpret_cast<uint4*>(c) = u;
        } else {
          for (int q = 0; q < 8 && n + q < g.N; ++q) c[q] = f32_to_bf16(v[q]);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();  // band reads done before the next band's writes
  }
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
// The K loop of one block tile (K-tiles kbase/BK .. +nk) into the wave's accumulators.
template <class T, int SCHED>
__device__ __forceinline__ void mainloop(f32x4_t (&acc)[T::FI][T::FJ], const BigGemmArgs& g, int m0, int n0, int nk,
                                         int kbase, uint8_t* smem, int wid, int lane, int wr, int wc, int fr,
                                         int fq) {
  const uint16_t* A = static_cast<const uint16_t*>(g.A);
  const uint16_t* Bt = static_cast<const uint16_t*>(g.Bt);
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
}

template <class T, int OUT, int SCHED>
__global__ void __launch_bounds__(T::NT) gemm_bf16_lds_kernel(BigGemmArgs g, int tm, int tn, int kt_per) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tile = xcd_remap(blockIdx.x, tm * tn);
  const int bm = tile / tn, bn = tile % tn;
  const int m0 = bm * T::BM, n0 = bn * T::BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / T::WN, wc = wid % T::WN;
  const int nk_all = g.K / BK;
  const int kt_begin = blockIdx.y * kt_per;
  const int nk = min(nk_all, kt_begin + kt_per) - kt_begin;  // >= 1 (host sizes the split)
  const int kbase = kt_begin * BK;
  const int fr = lane & 15, fq = lane >> 4;

  f32x4_t acc[T::FI][T::FJ];
  mainloop<T, SCHED>(acc, g, m0, n0, nk, kbase, smem, wid, lane, wr, wc, fr, fq);

  if constexpr (OUT == 2) {
    store_tile<T::FI, T::FJ, OUT>(g, acc, m0, n0, wr, wc, fr, fq);
  } else {
    __builtin_amdgcn_s_barrier();  // every wave's fragment reads done: the LDS is scratch now
    store_tile_lds<T::FI, T::FJ, OUT>(g, acc, m0, n0, wr, wc, fr, fq,
                                      reinterpret_cast<float*>(smem) + wid * epi_floats<T::FJ>());
  }
}

// ---------------------------------------------------------------------------------------------
// 1x1 convolution + BatchNorm statistics (ops/convbn.py): the bf16 GEMM above on the NHWC
// activation viewed as [M = N*H*W, Cin] against the [Cout, Cin] weight, whose epilogue also
// produces the training BatchNorm's per-channel batch statistics of the bf16 output -- the
// separate statistics pass over the conv output (one full read of it, bn_stats_kernel in
// batchnorm.hip) disappears.
//
//   1. each wave reduces its FI*16-row x FJ*16-column sub-tile from the accumulators
//      (bf16-rounded, exactly the stored values): per column the sum and the sum of squares
//      about the wave's own column mean (two passes over registers, lanes combined with
//      shuffles), written as one partial (row-disjoint, no atomics) per wave row;
//   2. groups of G row tiles per column tile: the last workgroup of a group to finish (atomic
//      ticket; partials handed over with sc1 stores/loads, see last_arrival) merges the group's partials in
//      fixed order (Chan et al.'s pairwise update, in double) into one group partial;
//   3. the last group of a column tile merges the group partials and writes mean, invstd,
//      scale = w*invstd, shift = b - mean*scale (the [4, C] layout batchnorm.hip's backward
//      reads), updates running_mean / running_var (unbiased) and num_batches_tracked.
// Deterministic (fixed merge order whatever the arrival order) and robust for |mean| >> std
// (centred partials). Tickets are re-armed by their last arriver for the next launch.
__device__ __forceinline__ float bf16_round(float v) { return bf16_to_f32(f32_to_bf16(v)); }

// (n, S, Q) <- (n, S, Q) merged with (np, Sp, Qp): S = sum, Q = sum of squares about the mean
__device__ __forceinline__ void chan_merge(double& n, double& S, double& Q, double np, double Sp, double Qp) {
  if (np <= 0.0) return;
  if (n <= 0.0) {
    n = np, S = Sp, Q = Qp;
    return;
  }
  const double d = Sp / np - S / n;
  Q += Qp + d * d * n * np / (n + np);
  S += Sp;
  n += np;
}

// Cross-workgroup hand-off of the statistics partials without L2 write-backs: every partial is
// stored and loaded with sc1 (write-through / L1-bypassing agent-scope relaxed atomics), every
// storing wave drains its stores (vmcnt(0)) before the workgroup barrier, then one lane adds to the
// ticket and the add's returned value names the last arriver (MI355X_MICROARCH.md "Hand-offs
// measured with sc1 loads", first row). An agent-scope release fence here would write back the
// XCD L2's dirty lines -- the freshly stored output tiles -- once per workgroup: +110 us on a
// 401408 x 256 conv (profiles/r3_convbn.md).
typedef __attribute__((address_space(1))) float gfloat;
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store((gfloat*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load((gfloat*)p, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// true in exactly one workgroup per ticket (the count-th arriver); re-arms the ticket
__device__ __forceinline__ bool last_arrival(int* ticket, int count, int* sh_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 partial stores have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == count - 1;
    if (last) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *sh_flag = last;
  }
  __syncthreads();
  // relaxed atomics carry no happens-before in the HIP model: visibility rests on the sc1 stores /
  // loads (see batchnorm.hip last_block); this fence keeps the partial loads below the ticket in the IR
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  return *sh_flag != 0;
}

// Merge partials [p0, p1) (row counts from rows_of(p)) of this tile's BN columns; the NT/BN thread
// groups take interleaved partials and are merged in group order through LDS. Result (n, S, Q)
// valid in threads t < BN.
template <class T, class RowsOf>
__device__ __forceinline__ void merge_range(const float* wsS, const float* wsQ, int N, int n0, int p0, int p1,
                                            RowsOf rows_of, double* sh, double& n, double& S, double& Q) {
  constexpr int PARTS = T::NT / T::BN;
  const int tid = threadIdx.x, col = tid % T::BN, part = tid / T::BN;
  const int c = n0 + col;
  n = S = Q = 0.0;
  if (c < N) {
    for (int p = p0 + part; p < p1; p += PARTS)
      chan_merge(n, S, Q, (double)rows_of(p), (double)ld_sc1(wsS + (int64_t)p * N + c),
                 (double)ld_sc1(wsQ + (int64_t)p * N + c));
  }
  __syncthreads();  // LDS scratch free
  if (part > 0) {
    sh[(part * 3 + 0) * T::BN + col] = n;
    sh[(part * 3 + 1) * T::BN + col] = S;
    sh[(part * 3 + 2) * T::BN + col] = Q;
  }
  __syncthreads();
  if (part == 0) {
#pragma unroll
    for (int q = 1; q < PARTS; ++q)
      chan_merge(n, S, Q, sh[(q * 3 + 0) * T::BN + col], sh[(q * 3 + 1) * T::BN + col],
                 sh[(q * 3 + 2) * T::BN + col]);
  }
}

template <class T, int SCHED>
__global__ void __launch_bounds__(T::NT) gemm_bn_stats_kernel(BigGemmArgs g, GemmBnEpi e, int tm, int tn) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tile = xcd_remap(blockIdx.x, tm * tn);
  const int bm = tile / tn, bn = tile % tn;
  const int m0 = bm * T::BM, n0 = bn * T::BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / T::WN, wc = wid % T::WN;
  const int fr = lane & 15, fq = lane >> 4;
  const int N = g.N;

  f32x4_t acc[T::FI][T::FJ];
  mainloop<T, SCHED>(acc, g, m0, n0, g.K / BK, 0, smem, wid, lane, wr, wc, fr, fq);

  // 1. wave partials: rows wrow0 .. wrow0 + FI*16 (nvalid of them inside M), columns of lane fr
  constexpr int WROWS = T::FI * 16;
  const int P = tm * T::WM;  // wave-row partials per column
  const int wrow0 = m0 + wr * WROWS;
  const int nvalid = max(0, min(g.M - wrow0, WROWS));
  float s[T::FJ], q[T::FJ];
#pragma unroll
  for (int j = 0; j < T::FJ; ++j) {
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < T::FI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (wrow0 + i * 16 + 4 * fq + r < g.M) a += bf16_round(acc[i][j][r]);
    a += __shfl_xor(a, 16);
    a += __shfl_xor(a, 32);
    s[j] = a;
  }
  const float inv_n = nvalid > 0 ? 1.f / (float)nvalid : 0.f;
#pragma unroll
  for (int j = 0; j < T::FJ; ++j) {
    const float mu = s[j] * inv_n;
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < T::FI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (wrow0 + i * 16 + 4 * fq + r < g.M) {
          const float d = bf16_round(acc[i][j][r]) - mu;
          a = fmaf(d, d, a);
        }
    a += __shfl_xor(a, 16);
    a += __shfl_xor(a, 32);
    q[j] = a;
  }
  float* wsS = e.ws;
  float* wsQ = e.ws + (int64_t)P * N;
  if (fq == 0) {
    const int p = bm * T::WM + wr;
#pragma unroll
    for (int j = 0; j < T::FJ; ++j) {
      const int c = n0 + wc * (T::FJ * 16) + j * 16 + fr;
      if (c < N) {
        st_sc1(wsS + (int64_t)p * N + c, s[j]);
        st_sc1(wsQ + (int64_t)p * N + c, q[j]);
      }
    }
  }

  // the bf16 output tile (coalesced through LDS)
  __builtin_amdgcn_s_barrier();  // every wave's fragment reads done: the LDS is scratch now
  store_tile_lds<T::FI, T::FJ, 0>(g, acc, m0, n0, wr, wc, fr, fq,
                                  reinterpret_cast<float*>(smem) + wid * epi_floats<T::FJ>());

  // 2. group merge by the group's last row tile
  double* sh = reinterpret_cast<double*>(smem);
  int* flag = reinterpret_cast<int*>(smem + 3 * T::NT * sizeof(double));
  const int G = e.group, ng = (tm + G - 1) / G;
  const int gi = bm / G;
  const int g_first = gi * G, g_count = min(G, tm - g_first);
  __syncthreads();  // epilogue scratch reads done before the LDS is reused
  if (!last_arrival(e.tickets + gi * tn + bn, g_count, flag)) return;
  double n, S, Q;
  auto wave_rows = [&](int p) { return max(0, min(g.M - (p / T::WM) * T::BM - (p % T::WM) * WROWS, WROWS)); };
  merge_range<T>(wsS, wsQ, N, n0, g_first * T::WM, (g_first + g_count) * T::WM, wave_rows, sh, n, S, Q);
  float* gS = e.ws + (int64_t)2 * P * N;
  float* gQ = gS + (int64_t)ng * N;
  {
    const int c = n0 + tid;
    if (tid < T::BN && c < N) {
      st_sc1(gS + (int64_t)gi * N + c, (float)S);
      st_sc1(gQ + (int64_t)gi * N + c, (float)Q);
    }
  }

  // 3. column-tile merge by the last group, final coefficients
  if (!last_arrival(e.tickets + ng * tn + bn, ng, flag)) return;
  const int64_t grows = (int64_t)G * T::BM;
  auto group_rows = [&](int p) { return (int)max((int64_t)0, min((int64_t)g.M - p * grows, grows)); };
  merge_range<T>(gS, gQ, N, n0, 0, ng, group_rows, sh, n, S, Q);
  const int c = n0 + tid;
  if (tid < T::BN && c < N) {
    const BnParams& p = e.p;
    const double Md = (double)g.M;
    const double mean = S / Md;
    const double var = Q / Md > 0.0 ? Q / Md : 0.0;
    const float invstd = (float)(1.0 / sqrt(var + (double)p.eps));
    const float w = p.weight ? p.weight[c] : 1.f, b = p.bias ? p.bias[c] : 0.f;
    p.mean[c] = (float)mean;
    p.invstd[c] = invstd;
    p.scale[c] = w * invstd;
    p.shift[c] = b - (float)mean * w * invstd;
    if (p.running_mean) {
      const double unbiased = g.M > 1 ? var * Md / (Md - 1.0) : var;
      p.running_mean[c] = (float)((1.0 - p.momentum) * p.running_mean[c] + p.momentum * mean);
      p.running_var[c] = (float)((1.0 - p.momentum) * p.running_var[c] + p.momentum * unbiased);
    }
  }
  if (tid == 0 && bn == 0 && e.p.num_batches_tracked) *e.p.num_batches_tracked += 1;
}


// SCHED 2 (256x256 geometry, BK = 64): the ping-pong pairs of SCHED 1 fed from a ring of ten
// 16-KiB operand pieces that fills the 160 KiB of LDS, so every DMA is issued 3-4 slots before
// its first reader (SCHED 1: 2) and no wait ever drains the queue in the loop.
//   pieces of K-tile t: A0 / A1 = A rows 0-127 / 128-255 (read by the leader wr = 0 in slot 2t /
//   the follower wr = 1 in slot 2t+1), B0 / B1 = B rows 0-127 / 128-255 (both groups).
//   issue schedule: slot 2k: A1(k+1), B0(k+2), B1(k+2); slot 2k+1: A0(k+2).
//   storage: A0(t) in one of two dedicated slots (t & 1: A0(t+2) is issued right after A0(t)'s
//   reader, the leader, is done); A1 / B0 / B1 in an 8-slot FIFO in issue order (position
//   3(t-1) for A1(t), 3(t-2) + 1 / + 2 for B0(t) / B1(t)), whose three oldest entries --
//   tile t-1's B0, B1, A1 -- are released together when the follower finishes tile t-1.
//   waits (per wave, its own LDS-DMAs, 2 per piece): before slot 2s the pieces B0, B1, A0 of
//   tile s are retired (at most 8 later DMAs in flight), before slot 2s+1 A1(s) is (at most 12).
constexpr int PIECE = 128 * BK * 2;  // 16 KiB
constexpr int PLDS = 10 * PIECE;     // 160 KiB
static_assert(8 * epi_floats<4>() * 4 <= PLDS, "epilogue scratch exceeds the LDS");

__device__ __forceinline__ int fifo_slot(int pos) { return (pos + 16) & 7; }

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N == 0 || N == 2 || N == 8 || N == 12, "add the literal");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
}

template <int OUT>
__global__ void __launch_bounds__(512) gemm_bf16_piece_kernel(BigGemmArgs g, int tm, int tn, int kt_per) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int FI = 8, FJ = 4;  // 128 x 64 per wave
  const int tile = xcd_remap(blockIdx.x, tm * tn);
  const int m0 = (tile / tn) * 256, n0 = (tile % tn) * 256;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const uint16_t* A = static_cast<const uint16_t*>(g.A);
  const uint16_t* Bt = static_cast<const uint16_t*>(g.Bt);
  const int nk_all = g.K / BK;
  const int kt_begin = blockIdx.y * kt_per;
  const int nk = min(nk_all, kt_begin + kt_per) - kt_begin;
  const int kbase = kt_begin * BK;
  const int fr = lane & 15, fq = lane >> 4;

  f32x4_t acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  auto a0_base = [&](int t) { return smem + (8 + (t & 1)) * PIECE; };
  auto a1_base = [&](int t) { return smem + fifo_slot(3 * (t - 1)) * PIECE; };
  auto b_base = [&](int t, int h) { return smem + fifo_slot(3 * (t - 2) + 1 + h) * PIECE; };
  auto stage_a = [&](int t, int h, uint8_t* dst) {
    stage_tile<128, 512>(A, g.lda, m0 + 128 * h, g.M, kbase + t * BK, dst, wid, lane);
  };
  auto stage_b = [&](int t, int h) {
    stage_tile<128, 512>(Bt, g.ldb, n0 + 128 * h, g.N, kbase + t * BK, b_base(t, h), wid, lane);
  };
  auto issue_slot = [&](int slot) {
    const int k = slot >> 1;
    if ((slot & 1) == 0) {
      if (k + 1 < nk) stage_a(k + 1, 1, a1_base(k + 1));
      if (k + 2 < nk) {
        stage_b(k + 2, 0);
        stage_b(k + 2, 1);
      }
    } else if (k + 2 < nk) {
      stage_a(k + 2, 0, a0_base(k + 2));
    }
  };
  // end of slot 2s: A1(s) retired; end of slot 2s+1: B0, B1, A0 of tile s+1 retired
  auto wait_even = [&](int s) {
    if (s + 2 < nk) vm_wait<12>();
    else if (s + 1 < nk) vm_wait<8>();
    else vm_wait<0>();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto wait_odd = [&](int s) {
    if (s + 2 < nk) vm_wait<8>();
    else if (s + 1 < nk) vm_wait<2>();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto slot_barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  bf16x8_t a[2][FI], b[2][FJ];
  auto read = [&](const uint8_t* ap, const uint8_t* bp) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int j = 0; j < FJ; ++j) b[kb][j] = read_frag(bp, (wc & 1) * 64 + j * 16 + fr, kb * 4 + fq);
#pragma unroll
      for (int i = 0; i < FI; ++i) a[kb][i] = read_frag(ap, i * 16 + fr, kb * 4 + fq);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mma = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kb][i], b[kb][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: B0(0), B1(0), A0(0), A1(0), B0(1), B1(1), A0(1) -- the issue order the waits count
  stage_b(0, 0);
  stage_b(0, 1);
  stage_a(0, 0, a0_base(0));
  stage_a(0, 1, a1_base(0));
  if (nk > 1) {
    stage_b(1, 0);
    stage_b(1, 1);
    stage_a(1, 0, a0_base(1));
    vm_wait<8>();
  } else {
    vm_wait<2>();
  }
  slot_barrier();
  if (wr == 0) {
    for (int s = 0; s < nk; ++s) {
      issue_slot(2 * s);
      read(a0_base(s), b_base(s, wc >> 1));
      wait_even(s);
      slot_barrier();
      issue_slot(2 * s + 1);
      mma();
      wait_odd(s);
      slot_barrier();
    }
  } else {
    for (int s = 0; s < nk; ++s) {
      issue_slot(2 * s);
      if (s > 0) mma();
      wait_even(s);
      slot_barrier();
      issue_slot(2 * s + 1);
      read(a1_base(s), b_base(s, wc >> 1));
      wait_odd(s);
      slot_barrier();
    }
    mma();
  }
  if constexpr (OUT == 2) {
    store_tile<FI, FJ, OUT>(g, acc, m0, n0, wr, wc, fr, fq);
  } else {
    __builtin_amdgcn_s_barrier();  // every wave's fragment reads done: the LDS is scratch now
    store_tile_lds<FI, FJ, OUT>(g, acc, m0, n0, wr, wc, fr, fq,
                                reinterpret_cast<float*>(smem) + wid * epi_floats<FJ>());
  }
}

template <int OUT>
hipError_t launch_piece(const BigGemmArgs& g, int split, hipStream_t s) {
  const void* fn = reinterpret_cast<const void*>(&gemm_bf16_piece_kernel<OUT>);
  static bool attr_set = false;
  if (!attr_set) {
    PTDT_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, PLDS));
    attr_set = true;
  }
  const int tm = (g.M + 255) / 256, tn = (g.N + 255) / 256;
  const int nk = g.K / BK;
  const int kt_per = (nk + split - 1) / split;
  split = (nk + kt_per - 1) / kt_per;
  hipLaunchKernelGGL((gemm_bf16_piece_kernel<OUT>), dim3(tm * tn, split), dim3(512), PLDS, s, g, tm, tn, kt_per);
  return hipGetLastError();
}

// SCHED 3 (256x256, BK = 64, 8 waves 2 (M) x 4 (N), 128 KiB LDS): the 8-phase schedule of
// cdna_hip_programming.md ("The 256^2 8-phase template"). Each K-tile is staged as four 16-KiB
// quarters (LDS-DMA, 2 per thread each), and each of its 4 phases computes one 64x32 quadrant of the
// wave's 128x64 output (16 MFMAs) between two barriers, after reading only that quadrant's new
// fragments -- the reads of the next quadrant, the DMA of one future quarter and the MFMAs of the
// current one interleave at phase granularity. The wr = 1 waves run one barrier behind the wr = 0
// waves (the SIMD's two waves alternate between LDS reads and MFMAs).
//   quarters (LDS slot: content; phase of its last read): 0: QA0 = A rows 64 s.. of each 128-row band
//   with s = 0 (phase 0), 1: QB1 = B rows 32..63 of each 64-row band (phase 1), 2: QA1 (phase 2),
//   3: QB0 (phase 0). Phases: 0 reads QA0 + QB0 -> quadrant (0, 0); 1 reads QB1 -> (0, 1); 2 reads QA1
//   -> (1, 1); 3 reads nothing -> (1, 0).
//   staging: global phase P = 4 t + r issues quarter (P + 7) & 3 of K-tile (P + 7) >> 2, i.e. 3
//   quarters ahead; a quarter is restaged one phase after its last read, which every wave retired
//   (lgkmcnt(0)) before that phase's first barrier; phase 3 waits (counted vmcnt, before its first
//   barrier) for the next K-tile, whose first reader starts a barrier later for both wave groups.
constexpr int QBYTES = 128 * BK * 2;  // 16 KiB quarter
constexpr int P8OPS = 8 * QBYTES;     // 2 K-tiles x 4 quarters: 128 KiB
constexpr int P8LDS = P8OPS > 8 * epi_floats<4>() * 4 ? P8OPS : 8 * epi_floats<4>() * 4;  // + epilogue: 136 KiB

__device__ __forceinline__ void vm_wait_n(int n) {
  if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// GRP > 0: tiles ordered in groups of GRP tile rows, column-major inside a group, so one XCD's
// contiguous chunk of the grid (xcd_remap) is a GRP x (chunk / GRP) block: its concurrently running
// workgroups share GRP A panels and a few B panels in that XCD's L2 instead of one A panel and ~32
// B panels (row-major order).
template <int GRP>
__device__ __forceinline__ void tile_coords(int tile, int tm, int tn, int& bm, int& bn) {
  if constexpr (GRP == 0) {
    bm = tile / tn;
    bn = tile % tn;
  } else {
    const int per = GRP * tn;
    const int grp = tile / per, first = grp * GRP;
    const int gsz = min(tm - first, GRP);
    const int in = tile - grp * per;
    bm = first + in % gsz;
    bn = in / gsz;
  }
}

template <int OUT, int GRP>
__global__ void __launch_bounds__(512) gemm_bf16_p8_kernel(BigGemmArgs g, int tm, int tn, int kt_per) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int FI = 8, FJ = 4;
  int bm, bn;
  tile_coords<GRP>(xcd_remap(blockIdx.x, tm * tn), tm, tn, bm, bn);
  const int m0 = bm * 256, n0 = bn * 256;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const uint16_t* A = static_cast<const uint16_t*>(g.A);
  const uint16_t* Bt = static_cast<const uint16_t*>(g.Bt);
  const int nk_all = g.K / BK;
  const int kt_begin = blockIdx.y * kt_per;
  const int nk = min(nk_all, kt_begin + kt_per) - kt_begin;
  const int kbase = kt_begin * BK;
  const int fr = lane & 15, fq = lane >> 4;
  const int H = 4 * nk;  // quarters to stage

  f32x4_t acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // quarter h = 4 k + q of K-tile k into slot (k & 1, q): rows of the quarter map to operand rows
  auto stage_q = [&](int h) {
    if (h >= H) return;
    const int k = h >> 2, q = h & 3;
    const bool isA = (q & 1) == 0;     // slots 0, 2: A quarters (s = q >> 1); 1, 3: B (s = 1 for q = 1)
    const int sub = isA ? (q >> 1) : (q == 1 ? 1 : 0);
    uint8_t* dst0 = smem + ((k & 1) * 4 + q) * QBYTES;
    const uint16_t* src = isA ? A : Bt;
    const int64_t ld = isA ? g.lda : g.ldb;
    const int nrows = isA ? g.M : g.N;
    const int k0 = kbase + k * BK;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int p = i * 512 + wid * 64 + lane;  // 16-B chunk of the quarter image
      const int r = p >> 3, slot = p & 7;
      const int c = slot ^ ((r >> 1) & 7);
      const int grow = isA ? m0 + 128 * (r >> 6) + 64 * sub + (r & 63) : n0 + 64 * (r >> 5) + 32 * sub + (r & 31);
      const uint16_t* gp = src + (int64_t)min(grow, nrows - 1) * ld + k0 + c * 8;
      __builtin_amdgcn_global_load_lds((gbl_void*)gp, (lds_void*)(dst0 + (i * 512 + wid * 64) * 16), 16, 0, 0);
    }
  };
  auto bar = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  bf16x8_t af[2][4], b0[2][2], b1[2][2];
  auto read_a = [&](const uint8_t* qa) {  // this wave's 64 rows of the quarter: band wr
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[kb][i] = read_frag(qa, 64 * wr + 16 * i + fr, kb * 4 + fq);
  };
  auto read_b = [&](bf16x8_t (&b)[2][2], const uint8_t* qb) {  // this wave's 32 columns: band wc
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int j = 0; j < 2; ++j) b[kb][j] = read_frag(qb, 32 * wc + 16 * j + fr, kb * 4 + fq);
  };
  auto mma = [&](int ia, const bf16x8_t (&b)[2][2], int jb) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[ia + i][jb + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kb][i], b[kb][j], acc[ia + i][jb + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: quarters 0..6 (K-tile 0 whole, K-tile 1's first three), K-tile 0 retired
  for (int h = 0; h < 7; ++h) stage_q(h);
  vm_wait_n(2 * (min(H, 7) - min(H, 4)));
  bar();
  if (wr == 1) bar();  // the wr = 1 waves run one barrier behind
  for (int t = 0; t < nk; ++t) {
    const uint8_t* bufb = smem + (t & 1) * 4 * QBYTES;
    // phase 0: QA0 + QB0 -> quadrant (0, 0)
    read_b(b0, bufb + 3 * QBYTES);
    read_a(bufb);
    stage_q(4 * t + 7);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    mma(0, b0, 0);
    bar();
    // phase 1: QB1 -> (0, 1)
    read_b(b1, bufb + 1 * QBYTES);
    stage_q(4 * t + 8);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    mma(0, b1, 2);
    bar();
    // phase 2: QA1 -> (1, 1)
    read_a(bufb + 2 * QBYTES);
    stage_q(4 * t + 9);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
    mma(4, b1, 2);
    bar();
    // phase 3: no reads -> (1, 0); K-tile t+1 retired before the first barrier
    stage_q(4 * t + 10);
    {
      const int issued = min(H, 4 * t + 11), need = min(H, 4 * t + 8);
      vm_wait_n(2 * (issued - need));
    }
    bar();
    mma(4, b0, 0);
    bar();
  }
  if (wr == 0) bar();  // balance the wr = 1 waves' extra barrier
  if constexpr (OUT == 2) {
    store_tile<FI, FJ, OUT>(g, acc, m0, n0, wr, wc, fr, fq);
  } else {
    __builtin_amdgcn_s_barrier();  // every wave's fragment reads done: the LDS is scratch now
    store_tile_lds<FI, FJ, OUT>(g, acc, m0, n0, wr, wc, fr, fq,
                                reinterpret_cast<float*>(smem) + wid * epi_floats<FJ>());
  }
}

template <int OUT, int GRP>
hipError_t launch_p8(const BigGemmArgs& g, int split, hipStream_t s) {
  const void* fn = reinterpret_cast<const void*>(&gemm_bf16_p8_kernel<OUT, GRP>);
  static bool attr_set = false;
  if (!attr_set) {
    PTDT_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, P8LDS));
    attr_set = true;
  }
  const int tm = (g.M + 255) / 256, tn = (g.N + 255) / 256;
  const int nk = g.K / BK;
  const int kt_per = (nk + split - 1) / split;
  split = (nk + kt_per - 1) / kt_per;
  hipLaunchKernelGGL((gemm_bf16_p8_kernel<OUT, GRP>), dim3(tm * tn, split), dim3(512), P8LDS, s, g, tm, tn, kt_per);
  return hipGetLastError();
}

// operand double buffer, or the coalesced epilogue's scratch if that is larger
template <class T>
constexpr int lds_bytes() {
  return T::LDS > (T::NT / 64) * epi_floats<T::FJ>() * 4 ? T::LDS : (T::NT / 64) * epi_floats<T::FJ>() * 4;
}

template <class T, int OUT, int SCHED>
hipError_t launch(const BigGemmArgs& g, int split, hipStream_t s) {
  const void* fn = reinterpret_cast<const void*>(&gemm_bf16_lds_kernel<T, OUT, SCHED>);
  constexpr int lds = lds_bytes<T>();
  static bool attr_set = false;  // one flag per instantiation
  if (!attr_set) {
    PTDT_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr_set = true;
  }
  const int tm = (g.M + T::BM - 1) / T::BM, tn = (g.N + T::BN - 1) / T::BN;
  const int nk = g.K / BK;
  const int kt_per = (nk + split - 1) / split;
  split = (nk + kt_per - 1) / kt_per;  // no empty slices
  hipLaunchKernelGGL((gemm_bf16_lds_kernel<T, OUT, SCHED>), dim3(tm * tn, split), dim3(T::NT), lds, s, g, tm, tn,
                     kt_per);
  return hipGetLastError();
}

template <class T, int SCHED>
hipError_t launch_out(const BigGemmArgs& g, int split, hipStream_t s) {
  if (split > 1) return launch<T, 2, SCHED>(g, split, s);
  return g.out_dtype == kF32 ? launch<T, 1, SCHED>(g, 1, s) : launch<T, 0, SCHED>(g, 1, s);
}

template <class T>
constexpr int bn_lds_bytes() {
  return lds_bytes<T>() > 3 * T::NT * 8 + 16 ? lds_bytes<T>() : 3 * T::NT * 8 + 16;
}

int bn_group(int tm) {
  int G = 1;
  while (G * G < tm) ++G;  // ceil(sqrt(tm)): group merges and the final merge read alike
  return G;
}

template <class T>
hipError_t launch_bn(const BigGemmArgs& g, GemmBnEpi e, hipStream_t s) {
  const void* fn = reinterpret_cast<const void*>(&gemm_bn_stats_kernel<T, T::NT == 512 ? 1 : 0>);
  constexpr int lds = bn_lds_bytes<T>();
  static bool attr_set = false;
  if (!attr_set) {
    PTDT_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    attr_set = true;
  }
  const int tm = (g.M + T::BM - 1) / T::BM, tn = (g.N + T::BN - 1) / T::BN;
  e.group = bn_group(tm);
  hipLaunchKernelGGL((gemm_bn_stats_kernel<T, T::NT == 512 ? 1 : 0>), dim3(tm * tn), dim3(T::NT), lds, s, g, e, tm,
                     tn);
  return hipGetLastError();
}

}  // namespace

int64_t gemm_bn_ws_floats(int M, int N, int tile) {
  const int bm = tile == 128 ? 128 : 256, wm = 2;
  const int tm = (M + bm - 1) / bm;
  const int ng = (tm + bn_group(tm) - 1) / bn_group(tm);
  return (int64_t)2 * N * ((int64_t)tm * wm + ng);
}

int gemm_bn_num_tickets(int M, int N, int tile) {
  const int bm = tile == 128 ? 128 : 256;
  const int tm = (M + bm - 1) / bm, tn = (N + bm - 1) / bm;
  const int ng = (tm + bn_group(tm) - 1) / bn_group(tm);
  return (ng + 1) * tn;
}

hipError_t gemm_bn_stats(const BigGemmArgs& g, GemmBnEpi e, hipStream_t s) {
  if (!gemm_bf16_big_supported(g.M, g.N, g.K, g.lda, g.ldb, g.A, g.Bt)) return hipErrorInvalidValue;
  if (g.out_dtype != kBF16 || g.split_k > 1 || g.ldc % 8 != 0 || e.ws == nullptr || e.tickets == nullptr ||
      e.p.mean == nullptr || e.p.invstd == nullptr || e.p.scale == nullptr || e.p.shift == nullptr)
    return hipErrorInvalidValue;
  BigGemmArgs a = g;
  a.alpha = 1.f, a.beta = 0.f, a.relu = 0, a.bias = nullptr;
  if (g.tile == 128) return launch_bn<T128>(a, e, s);
  if (g.tile == 256) return launch_bn<T256>(a, e, s);
  return hipErrorInvalidValue;
}

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
  static_assert(lds_bytes<T256>() <= 160 * 1024 && 2 * lds_bytes<T128>() <= 160 * 1024, "LDS budget");
  if (g.sched == 0) return launch_out<T256, 0>(g, split, s);
  if (g.sched == 1) return launch_out<T256, 1>(g, split, s);
  if (g.sched == 2) {
    if (split > 1) return launch_piece<2>(g, split, s);
    return g.out_dtype == kF32 ? launch_piece<1>(g, 1, s) : launch_piece<0>(g, 1, s);
  }
  if (g.sched == 3) {
    if (split > 1) return launch_p8<2, 0>(g, split, s);
    return g.out_dtype == kF32 ? launch_p8<1, 0>(g, 1, s) : launch_p8<0, 0>(g, 1, s);
  }
  if (g.sched == 4) {  // 8-phase with grouped tile order (8 tile rows per group)
    if (split > 1) return launch_p8<2, 8>(g, split, s);
    return g.out_dtype == kF32 ? launch_p8<1, 8>(g, 1, s) : launch_p8<0, 8>(g, 1, s);
  }
  if (g.sched == 5) {  // group of 4 tile rows (A/B of the group size)
    if (split > 1) return launch_p8<2, 4>(g, split, s);
    return g.out_dtype == kF32 ? launch_p8<1, 4>(g, 1, s) : launch_p8<0, 4>(g, 1, s);
  }
  if (g.sched == 6) {  // group of 16 tile rows
    if (split > 1) return launch_p8<2, 16>(g, split, s);
    return g.out_dtype == kF32 ? launch_p8<1, 16>(g, 1, s) : launch_p8<0, 16>(g, 1, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace ptdt
