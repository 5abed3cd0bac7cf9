// Large-shape bf16 GEMM for gfx950: 256x256x64 block tile, LDS-DMA staging,
// double-buffered, XCD-aware tile order, Linear-layer epilogue fused.
//
//   C[M,N] = alpha * A[M,K] . Bt[N,K]^T (+ beta*C) (+ bias[N]) (ReLU)
//
// Both operands are K-contiguous (row-major A, and B given as its transpose
// Bt[N,K] -- exactly nn.Linear's weight layout, so y = x W^T needs no copy).
// This is the throughput path of ops/linear.py for big shapes; the strided
// 64x64 kernel in gemm.hip keeps the odd layouts and fusions (ReLU mask on A,
// bias-grad row sums, split-K) for the small and latency-bound ones.
//
// Structure (cdna_hip_programming.md §5, "glds, 2 LDS buffers, BK=64"):
//   * 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns a 128x64 output
//     sub-tile = 8x4 v_mfma_f32_16x16x32_bf16 accumulators (128 acc VGPRs).
//   * global -> LDS with global_load_lds_dwordx4 (16 B per lane, no VGPR
//     round trip): each wave-instruction fills 1 KiB of LDS linearly, so the
//     bank swizzle is applied to the per-lane SOURCE address and undone on the
//     ds_read side (same involution on both sides).
//   * swizzle: a 256x64 bf16 tile is 256 rows x 8 chunks of 16 B; chunk c of
//     row r lives in slot c ^ ((r >> 1) & 7). The 16 lanes of a ds_read_b128
//     (16 consecutive rows, same logical chunk) then hit 16 distinct 16-B slots
//     of one 256-B bank row: conflict-free.
//   * pipeline: tile k+1 is in flight (its LDS-DMA counted on vmcnt) while tile
//     k is multiplied; a counted `s_waitcnt vmcnt(8)` + raw s_barrier retires
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

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NT = 512;                       // 8 waves
constexpr int TILE_BYTES = BM * BK * 2;       // 32 KiB per operand tile
constexpr int BUF_BYTES = 2 * TILE_BYTES;     // A + B
constexpr int LDS_BYTES = 2 * BUF_BYTES;      // double buffered: 128 KiB
constexpr int GLDS_PER_TILE = TILE_BYTES / (NT * 16);  // 4 per thread per operand

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;

// Issue the LDS-DMA of one 256x64 operand tile (rows row0.., k0..k0+63) with THREADS threads.
template <int THREADS = NT>
__device__ __forceinline__ void stage_tile(const uint16_t* __restrict__ src, int64_t ld, int row0, int nrows,
                                           int k0, uint8_t* lds_tile, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < TILE_BYTES / (THREADS * 16); ++i) {
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

__device__ __forceinline__ bf16x8_t read_frag(const uint8_t* lds_tile, int row, int c) {
  const int slot = c ^ ((row >> 1) & 7);
  return *reinterpret_cast<const bf16x8_t*>(lds_tile + row * (BK * 2) + slot * 16);
}

// Fragment reads of one 64-deep K-tile for a wave's 128x64 sub-tile (24 x ds_read_b128).
struct Frags {
  bf16x8_t a[2][8], b[2][4];
};

__device__ __forceinline__ void read_tile(Frags& f, const uint8_t* at, const uint8_t* bt, int wr, int wc, int fr,
                                          int fq) {
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
    for (int j = 0; j < 4; ++j) f.b[kb][j] = read_frag(bt, wc * 64 + j * 16 + fr, kb * 4 + fq);
#pragma unroll
    for (int i = 0; i < 8; ++i) f.a[kb][i] = read_frag(at, wr * 128 + i * 16 + fr, kb * 4 + fq);
  }
}

__device__ __forceinline__ void mfma_tile(f32x4_t (&acc)[8][4], const Frags& f) {
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[kb][i], f.b[kb][j], acc[i][j], 0, 0, 0);
}

// SCHED 0: every wave reads then multiplies each K-tile (two barriers per tile,
//          tile k+1's DMA in flight meanwhile).
// SCHED 1: ping-pong. The two waves sharing a SIMD (wave w and w+4: the M-halves
//          wr = 0 / 1) run half a tile apart: while one multiplies K-tile t from
//          registers, its partner reads K-tile t's fragments from LDS, so the
//          SIMD's matrix pipe always has one wave feeding it. Slots are separated
//          by workgroup barriers; wr=1 waves start one slot late. Tile t+1's
//          DMA is issued at the start of slot 2t and retired (vmcnt(0)) before
//          the barrier closing slot 2t+1: its buffer's previous tile (t-1) was
//          last read in slot 2t-1, and its first reader starts in slot 2t+2.
template <bool OUT_F32, int SCHED>
__global__ void __launch_bounds__(NT, 1) gemm_bf16_256_kernel(BigGemmArgs g, int tm, int tn) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tile = xcd_remap(blockIdx.x, tm * tn);
  const int bm = tile / tn, bn = tile % tn;
  const int m0 = bm * BM, n0 = bn * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const uint16_t* A = static_cast<const uint16_t*>(g.A);
  const uint16_t* Bt = static_cast<const uint16_t*>(g.Bt);
  const int nk = g.K / BK;
  const int fr = lane & 15, fq = lane >> 4;

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  stage_tile(A, g.lda, m0, g.M, 0, smem, wid, lane);
  stage_tile(Bt, g.ldb, n0, g.N, 0, smem + TILE_BYTES, wid, lane);

  if constexpr (SCHED == 0) {
    for (int kt = 0; kt < nk; ++kt) {
      uint8_t* cur = smem + (kt & 1) * BUF_BYTES;
      if (kt + 1 < nk) {
        uint8_t* nxt = smem + ((kt + 1) & 1) * BUF_BYTES;
        stage_tile(A, g.lda, m0, g.M, (kt + 1) * BK, nxt, wid, lane);
        stage_tile(Bt, g.ldb, n0, g.N, (kt + 1) * BK, nxt + TILE_BYTES, wid, lane);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile kt landed, kt+1 still in flight
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();  // every wave's DMA of tile kt is visible
      __builtin_amdgcn_sched_barrier(0);
      Frags f;
      read_tile(f, cur, cur + TILE_BYTES, wr, wc, fr, fq);
      mfma_tile(acc, f);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();  // buffer kt&1 free for tile kt+2
    }
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // tile 0 visible
    __builtin_amdgcn_sched_barrier(0);
    Frags f;
    // one loop per role (same barrier count): the register allocator then
    // sees the fragments live only between their read and their MFMAs
    if (wr == 0) {  // leader: slot 2kt reads tile kt, slot 2kt+1 multiplies it
      for (int kt = 0; kt < nk; ++kt) {
        const uint8_t* cur = smem + (kt & 1) * BUF_BYTES;
        if (kt + 1 < nk) {
          uint8_t* nxt = smem + ((kt + 1) & 1) * BUF_BYTES;
          stage_tile(A, g.lda, m0, g.M, (kt + 1) * BK, nxt, wid, lane);
          stage_tile(Bt, g.ldb, n0, g.N, (kt + 1) * BK, nxt + TILE_BYTES, wid, lane);
        }
        read_tile(f, cur, cur + TILE_BYTES, wr, wc, fr, fq);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        mfma_tile(acc, f);
        __builtin_amdgcn_s_setprio(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile kt+1 landed (own DMA)
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {  // follower: slot 2kt multiplies tile kt-1, slot 2kt+1 reads tile kt
      for (int kt = 0; kt < nk; ++kt) {
        const uint8_t* cur = smem + (kt & 1) * BUF_BYTES;
        if (kt + 1 < nk) {
          uint8_t* nxt = smem + ((kt + 1) & 1) * BUF_BYTES;
          stage_tile(A, g.lda, m0, g.M, (kt + 1) * BK, nxt, wid, lane);
          stage_tile(Bt, g.ldb, n0, g.N, (kt + 1) * BK, nxt + TILE_BYTES, wid, lane);
        }
        if (kt > 0) {
          __builtin_amdgcn_s_setprio(1);
          mfma_tile(acc, f);
          __builtin_amdgcn_s_setprio(0);
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        read_tile(f, cur, cur + TILE_BYTES, wr, wc, fr, fq);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
      mfma_tile(acc, f);
    }
  }

  // epilogue: acc[i][j][r] = C[m0 + wr*128 + i*16 + 4*fq + r][n0 + wc*64 + j*16 + fr]
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wc * 64 + j * 16 + fr;
    if (n >= g.N) continue;
    float bias = 0.f;
    if (g.bias != nullptr)
      bias = g.bias_dtype == kF32 ? static_cast<const float*>(g.bias)[n]
                                  : bf16_to_f32(static_cast<const uint16_t*>(g.bias)[n]);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * 128 + i * 16 + 4 * fq + r;
        if (m >= g.M) continue;
        const int64_t off = (int64_t)m * g.ldc + n;
        float v = g.alpha * acc[i][j][r];
        if constexpr (OUT_F32) {
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

}  // namespace

bool gemm_bf16_big_supported(int M, int N, int K, int64_t lda, int64_t ldb, const void* A, const void* Bt) {
  return M > 0 && N > 0 && K >= BK && K % BK == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         (reinterpret_cast<uintptr_t>(A) & 15) == 0 && (reinterpret_cast<uintptr_t>(Bt) & 15) == 0;
}

hipError_t gemm_bf16_big(const BigGemmArgs& g, hipStream_t s) {
  if (!gemm_bf16_big_supported(g.M, g.N, g.K, g.lda, g.ldb, g.A, g.Bt)) return hipErrorInvalidValue;
  const int tm = (g.M + BM - 1) / BM, tn = (g.N + BN - 1) / BN;
  const int sched = g.sched;
  if (sched < 0 || sched > 1) return hipErrorInvalidValue;
  const void* fns[2][2] = {{reinterpret_cast<const void*>(&gemm_bf16_256_kernel<false, 0>),
                            reinterpret_cast<const void*>(&gemm_bf16_256_kernel<false, 1>)},
                           {reinterpret_cast<const void*>(&gemm_bf16_256_kernel<true, 0>),
                            reinterpret_cast<const void*>(&gemm_bf16_256_kernel<true, 1>)}};
  static bool attr_set[2][2] = {};
  const int which = g.out_dtype == kF32 ? 1 : 0;
  if (!attr_set[which][sched]) {
    PTDT_HIP_CHECK(hipFuncSetAttribute(fns[which][sched], hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
    attr_set[which][sched] = true;
  }
  const dim3 grid(tm * tn), block(NT);
  if (which) {
    if (sched == 1) hipLaunchKernelGGL((gemm_bf16_256_kernel<true, 1>), grid, block, LDS_BYTES, s, g, tm, tn);
    else hipLaunchKernelGGL((gemm_bf16_256_kernel<true, 0>), grid, block, LDS_BYTES, s, g, tm, tn);
  } else {
    if (sched == 1) hipLaunchKernelGGL((gemm_bf16_256_kernel<false, 1>), grid, block, LDS_BYTES, s, g, tm, tn);
    else hipLaunchKernelGGL((gemm_bf16_256_kernel<false, 0>), grid, block, LDS_BYTES, s, g, tm, tn);
  }
  return hipGetLastError();
}

}  // namespace ptdt
