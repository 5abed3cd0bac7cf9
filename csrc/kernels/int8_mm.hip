// LLM.int8 matrix multiply for gfx950: vector-wise int8 quantisation with the
// outlier decomposition of bitsandbytes (reference: BitsAndBytesConfig(load_in_8bit=True),
// NB03:52-56).
//
//   y = (Xq . Wq^T) * sx[m] * sw[n]  +  X[:, O] . Wdq[:, O]^T  (+ bias)
//
// O = the input features with |x| > threshold somewhere in the batch (column absmax);
// those columns are zeroed before the activation rows are quantised (absmax per row)
// and multiplied in 16/32-bit instead (the caller gathers them: usually a handful).
//   int8_col_outliers : column absmax > threshold -> mask[K] (row-chunked, atomic max)
//   int8_quant_rows   : per-row absmax over the non-outlier columns, q = rint(x / s)
//   int8_mm           : int32 products on v_mfma_i32_16x16x64_i8 (exact), dequantised in
//                       the fp32 epilogue with the addend (outlier part) and bias
// Activations / outputs / bias: fp32, bf16 or fp16 (the reference's Llama runs in fp16).
//
// int8_mm, tiled path (K % 128 == 0): 128x128 output tile per workgroup of 4 waves (2x2,
// 64x64 each = 4x4 MFMA tiles), K in 128-byte tiles staged global -> LDS with
// global_load_lds_dwordx4 (16 B per lane, no VGPR round trip), double-buffered: tile k+1's
// DMA is in flight (counted vmcnt) while tile k is multiplied. A tile is rows x 8 chunks
// of 16 B; chunk c of row r lives in slot c ^ ((r >> 1) & 7), so the 16 rows read by one
// ds_read_b128 hit 16 distinct slots (conflict-free) -- the layout of gemm_big.hip's bf16
// tiles, whose 64-element K-tile is the same 128 bytes. Workgroup ids are XCD-remapped.
// Shapes with >= 256 256x256 tiles take the 8-wave 256x256 ping-pong variant (i8_mm_t256_kernel).
// Direct path (other K % 16 == 0): fragments straight from global memory, 64x64 tiles.
#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

using i32x4 = __attribute__((ext_vector_type(4))) int;
constexpr int kThreads = 256;

// Column absmax over a chunk of rows: thread = one column (coalesced rows), grid (column
// blocks, row chunks); chunk maxima meet in amax[K] through an atomic max on the float bits
// (order-preserving for non-negative floats). Round 2 ran one thread per column over ALL
// rows: K / 256 workgroups (16 for K = 4096) and 5x the int8 GEMM's time.
constexpr int kRowsPerChunk = 64;
template <typename T>
__global__ void __launch_bounds__(kThreads) col_absmax_kernel(const T* __restrict__ x, int M, int K,
                                                              unsigned* __restrict__ amax_bits) {
  const int k = blockIdx.x * kThreads + threadIdx.x;
  if (k >= K) return;
  const int m0 = blockIdx.y * kRowsPerChunk, m1 = min(M, m0 + kRowsPerChunk);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;  // 4 loads in flight
  int m = m0;
  for (; m + 3 < m1; m += 4) {
    a0 = fmaxf(a0, fabsf(Cvt<T>::load(x, (int64_t)m * K + k)));
    a1 = fmaxf(a1, fabsf(Cvt<T>::load(x, (int64_t)(m + 1) * K + k)));
    a2 = fmaxf(a2, fabsf(Cvt<T>::load(x, (int64_t)(m + 2) * K + k)));
    a3 = fmaxf(a3, fabsf(Cvt<T>::load(x, (int64_t)(m + 3) * K + k)));
  }
  for (; m < m1; ++m) a0 = fmaxf(a0, fabsf(Cvt<T>::load(x, (int64_t)m * K + k)));
  const float a = fmaxf(fmaxf(a0, a1), fmaxf(a2, a3));
  atomicMax(amax_bits + k, __float_as_uint(a));
}

__global__ void __launch_bounds__(kThreads) col_mask_kernel(const unsigned* __restrict__ amax_bits, int K, float thr,
                                                            uint8_t* __restrict__ mask) {
  const int k = blockIdx.x * kThreads + threadIdx.x;
  if (k < K) mask[k] = __uint_as_float(amax_bits[k]) > thr ? 1 : 0;
}

template <typename T>
__global__ void __launch_bounds__(kThreads) row_quant_kernel(const T* __restrict__ x, int K,
                                                             const uint8_t* __restrict__ mask, int8_t* __restrict__ q,
                                                             float* __restrict__ scale) {
  __shared__ float red[16];
  const int64_t r = blockIdx.x;
  const T* xr = x + r * K;
  float amax = 0.f;
  for (int k = threadIdx.x; k < K; k += kThreads)
    if (!(mask && mask[k])) amax = fmaxf(amax, fabsf(Cvt<T>::load(xr, k)));
  amax = block_max(amax, red);
  const float sc = amax > 0.f ? amax / 127.f : 1.f;
  for (int k = threadIdx.x; k < K; k += kThreads) {
    float v = (mask && mask[k]) ? 0.f : rintf(Cvt<T>::load(xr, k) / sc);  // IEEE division, as the reference
    v = fminf(fmaxf(v, -127.f), 127.f);
    q[r * K + k] = (int8_t)v;
  }
  if (threadIdx.x == 0) scale[r] = sc;
}

__device__ __forceinline__ float load_any(const void* p, int dtype, int64_t i) {
  if (dtype == kF32) return static_cast<const float*>(p)[i];
  if (dtype == kF16) return (float)static_cast<const _Float16*>(p)[i];
  return bf16_to_f32(static_cast<const uint16_t*>(p)[i]);
}
__device__ __forceinline__ void store_any(void* p, int dtype, int64_t i, float v) {
  if (dtype == kF32) static_cast<float*>(p)[i] = v;
  else if (dtype == kF16) static_cast<_Float16*>(p)[i] = (_Float16)v;
  else static_cast<uint16_t*>(p)[i] = f32_to_bf16(v);
}

struct I8Epi {
  const float* sa;
  const float* sb;
  const float* addend;
  const void* bias;
  int bias_dtype;
  void* y;
  int y_dtype;
  int M, N;
};

// acc[i][j][r] = C[m0 + 16 i + 4 g + r][n0 + 16 j + c] of this wave's FI x FJ 16x16 tiles
template <int FI, int FJ>
__device__ __forceinline__ void i8_epilogue(const I8Epi& e, const i32x4 (&acc)[FI][FJ], int m0, int n0, int c,
                                            int g) {
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    const int n = n0 + 16 * j + c;
    if (n >= e.N) continue;
    const float sbn = e.sb[n];
    const float bn = e.bias ? load_any(e.bias, e.bias_dtype, n) : 0.f;
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + 16 * i + 4 * g + r;
        if (m >= e.M) continue;
        const int64_t off = (int64_t)m * e.N + n;
        float v = (float)acc[i][j][r] * e.sa[m] * sbn;
        if (e.addend) v += e.addend[off];
        v += bn;
        store_any(e.y, e.y_dtype, off, v);
      }
  }
}

// ------------------------------------------------------------------ direct path
// 64x64 output tile per workgroup, 4 waves of 32x32 (2x2 MFMA tiles of 16x16), K in steps of 64
__global__ void __launch_bounds__(kThreads) i8_mm_kernel(const int8_t* __restrict__ A, const int8_t* __restrict__ B,
                                                         int K, I8Epi e, int tm, int tn) {
  const int tile = xcd_remap(blockIdx.x, tm * tn);
  const int m0 = (tile / tn) * 64, n0 = (tile % tn) * 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int c = lane & 15, g = lane >> 4;
  i32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = i32x4{0, 0, 0, 0};
  int ra[2], rb[2];
  bool va[2], vb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    ra[i] = m0 + wr * 32 + 16 * i + c;
    va[i] = ra[i] < e.M;
    rb[i] = n0 + wc * 32 + 16 * i + c;
    vb[i] = rb[i] < e.N;
  }
  for (int k0 = 0; k0 < K; k0 += 64) {
    const int k = k0 + 16 * g;  // this lane group's 16 consecutive k (same set for A and B)
    const bool kin = k < K;
    i32x4 a[2], b[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      a[i] = (va[i] && kin) ? *reinterpret_cast<const i32x4*>(A + (int64_t)ra[i] * K + k) : i32x4{0, 0, 0, 0};
      b[i] = (vb[i] && kin) ? *reinterpret_cast<const i32x4*>(B + (int64_t)rb[i] * K + k) : i32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  i8_epilogue<2, 2>(e, acc, m0 + wr * 32, n0 + wc * 32, c, g);
}

// ------------------------------------------------------------------ tiled path
constexpr int TM = 128, TN = 128, BKB = 128;         // output tile, K bytes per K-tile
constexpr int TILE_BYTES = TM * BKB;                  // one operand tile (16 KiB)
constexpr int BUF = 2 * TILE_BYTES;                   // A + B
constexpr int LDS_BYTES = 2 * BUF;                    // double buffered: 64 KiB (2 workgroups per CU)

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;

// LDS-DMA of one ROWS x 128-byte operand tile (rows row0.., bytes k0..k0+127) by THREADS threads
template <int ROWS, int THREADS>
__device__ __forceinline__ void stage_i8(const int8_t* __restrict__ src, int K, int row0, int nrows, int k0,
                                         uint8_t* lds_tile, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < ROWS * BKB / (THREADS * 16); ++i) {
    const int p = i * THREADS + wid * 64 + lane;  // linear 16-B chunk of the tile image
    const int r = p >> 3, slot = p & 7;
    const int ch = slot ^ ((r >> 1) & 7);       // logical 16-B k-chunk stored in this slot
    const int gr = min(row0 + r, nrows - 1);    // clamp: edge rows are computed, never stored
    const int8_t* gsrc = src + (int64_t)gr * K + k0 + ch * 16;
    uint8_t* dst = lds_tile + (i * THREADS + wid * 64) * 16;  // wave-uniform base; hardware adds lane * 16
    __builtin_amdgcn_global_load_lds((gbl_void*)gsrc, (lds_void*)dst, 16, 0, 0);
  }
}

__device__ __forceinline__ i32x4 frag(const uint8_t* lds_tile, int row, int ch) {
  const int slot = ch ^ ((row >> 1) & 7);
  return *reinterpret_cast<const i32x4*>(lds_tile + row * BKB + slot * 16);
}

__global__ void __launch_bounds__(kThreads) i8_mm_tiled_kernel(const int8_t* __restrict__ A,
                                                               const int8_t* __restrict__ B, int K, I8Epi e, int tm,
                                                               int tn) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int FI = 4, FJ = 4;  // 64x64 per wave
  const int tile = xcd_remap(blockIdx.x, tm * tn);
  const int m0 = (tile / tn) * TM, n0 = (tile % tn) * TN;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int c = lane & 15, g = lane >> 4;
  const int nk = K / BKB;
  i32x4 acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = i32x4{0, 0, 0, 0};

  auto stage = [&](int kt, uint8_t* buf) {
    stage_i8<TM, kThreads>(A, K, m0, e.M, kt * BKB, buf, wid, lane);
    stage_i8<TN, kThreads>(B, K, n0, e.N, kt * BKB, buf + TILE_BYTES, wid, lane);
  };
  stage(0, smem);
  for (int kt = 0; kt < nk; ++kt) {
    const uint8_t* cur = smem + (kt & 1) * BUF;
    if (kt + 1 < nk) {
      stage(kt + 1, smem + ((kt + 1) & 1) * BUF);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile kt landed (2 x 4 DMAs), kt+1 in flight
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // every wave's DMA of tile kt is visible
    __builtin_amdgcn_sched_barrier(0);
    i32x4 a[2][FI], b[2][FJ];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {  // two 64-byte halves of the K-tile
#pragma unroll
      for (int j = 0; j < FJ; ++j) b[kb][j] = frag(cur + TILE_BYTES, wc * 64 + 16 * j + c, kb * 4 + g);
#pragma unroll
      for (int i = 0; i < FI; ++i) a[kb][i] = frag(cur, wr * 64 + 16 * i + c, kb * 4 + g);
    }
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[kb][i], b[kb][j], acc[i][j], 0, 0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();  // buffer kt & 1 free for tile kt + 2
  }
  i8_epilogue<FI, FJ>(e, acc, m0 + wr * 64, n0 + wc * 64, c, g);
}

// 256x256 tile, 8 waves (2 M x 4 N, 128x64 each = 8x4 MFMA tiles), 128 KiB LDS (one workgroup
// per CU), ping-pong wave pairs as gemm_big.hip's SCHED 1: the two waves sharing a SIMD (w and
// w + 4, M halves wr = 0 / 1) run half a K-tile apart, so while one multiplies from registers
// its partner reads the next fragments from LDS and the SIMD's matrix pipe stays fed. Tile
// t+1's DMA is issued at the start of slot 2t and retired (vmcnt(0)) before the barrier that
// closes slot 2t+1.
constexpr int TB = 256, TB_TILE = TB * BKB, TB_BUF = 2 * TB_TILE, TB_LDS = 2 * TB_BUF;  // 128 KiB
__global__ void __launch_bounds__(512) i8_mm_t256_kernel(const int8_t* __restrict__ A, const int8_t* __restrict__ B,
                                                         int K, I8Epi e, int tm, int tn) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int FI = 8, FJ = 4;
  const int tile = xcd_remap(blockIdx.x, tm * tn);
  const int m0 = (tile / tn) * TB, n0 = (tile % tn) * TB;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int c = lane & 15, g = lane >> 4;
  const int nk = K / BKB;
  i32x4 acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = i32x4{0, 0, 0, 0};
  auto stage = [&](int kt, uint8_t* buf) {
    stage_i8<TB, 512>(A, K, m0, e.M, kt * BKB, buf, wid, lane);
    stage_i8<TB, 512>(B, K, n0, e.N, kt * BKB, buf + TB_TILE, wid, lane);
  };
  i32x4 a[2][FI], b[2][FJ];
  auto read = [&](const uint8_t* cur) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int j = 0; j < FJ; ++j) b[kb][j] = frag(cur + TB_TILE, wc * 64 + 16 * j + c, kb * 4 + g);
#pragma unroll
      for (int i = 0; i < FI; ++i) a[kb][i] = frag(cur, wr * 128 + 16 * i + c, kb * 4 + g);
    }
  };
  auto mma = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[kb][i], b[kb][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto bar = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  stage(0, smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();  // tile 0 visible
  if (wr == 0) {  // leader: slot 2kt reads tile kt, slot 2kt+1 multiplies it
    for (int kt = 0; kt < nk; ++kt) {
      const uint8_t* cur = smem + (kt & 1) * TB_BUF;
      if (kt + 1 < nk) stage(kt + 1, smem + ((kt + 1) & 1) * TB_BUF);
      read(cur);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bar();
      mma();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile kt+1 landed (own DMAs)
      bar();
    }
  } else {  // follower: slot 2kt multiplies tile kt-1, slot 2kt+1 reads tile kt
    for (int kt = 0; kt < nk; ++kt) {
      const uint8_t* cur = smem + (kt & 1) * TB_BUF;
      if (kt + 1 < nk) stage(kt + 1, smem + ((kt + 1) & 1) * TB_BUF);
      if (kt > 0) mma();
      bar();
      read(cur);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
    }
    mma();
  }
  i8_epilogue<FI, FJ>(e, acc, m0 + wr * 128, n0 + wc * 64, c, g);
}

__global__ void __launch_bounds__(kThreads) zero_u32_kernel(unsigned* p, int n) {
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i < n) p[i] = 0u;
}

template <typename T>
hipError_t outliers_t(const void* x, int M, int K, float threshold, uint8_t* mask, unsigned* ws, hipStream_t s) {
  // zeroed by a kernel, not hipMemsetAsync: graph-replayed memset nodes are unreliable once eager
  // memsets run between replays (profiles/r4_graph_memset.md)
  const int cb = (K + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(zero_u32_kernel, dim3(cb), dim3(kThreads), 0, s, ws, K);
  if (M > 0) {
    const dim3 grid(cb, (M + kRowsPerChunk - 1) / kRowsPerChunk);
    hipLaunchKernelGGL(col_absmax_kernel<T>, grid, dim3(kThreads), 0, s, static_cast<const T*>(x), M, K, ws);
    PTDT_HIP_CHECK(hipGetLastError());
  }
  hipLaunchKernelGGL(col_mask_kernel, dim3(cb), dim3(kThreads), 0, s, ws, K, threshold, mask);
  return hipGetLastError();
}

template <typename T>
hipError_t quant_t(const void* x, int M, int K, const uint8_t* mask, int8_t* q, float* scale, hipStream_t s) {
  hipLaunchKernelGGL(row_quant_kernel<T>, dim3(M), dim3(kThreads), 0, s, static_cast<const T*>(x), K, mask, q, scale);
  return hipGetLastError();
}

}  // namespace

hipError_t int8_col_outliers(const void* x, int dtype, int M, int K, float threshold, uint8_t* mask, unsigned* ws,
                             hipStream_t s) {
  if (K <= 0) return hipSuccess;
  if (dtype == kF32) return outliers_t<float>(x, M, K, threshold, mask, ws, s);
  if (dtype == kF16) return outliers_t<_Float16>(x, M, K, threshold, mask, ws, s);
  return outliers_t<uint16_t>(x, M, K, threshold, mask, ws, s);
}

hipError_t int8_quant_rows(const void* x, int dtype, int M, int K, const uint8_t* mask, int8_t* q, float* scale,
                           hipStream_t s) {
  if (M <= 0 || K <= 0) return hipSuccess;
  if (dtype == kF32) return quant_t<float>(x, M, K, mask, q, scale, s);
  if (dtype == kF16) return quant_t<_Float16>(x, M, K, mask, q, scale, s);
  return quant_t<uint16_t>(x, M, K, mask, q, scale, s);
}

bool int8_mm_tiled_supported(int M, int N, int K) { return M > 0 && N > 0 && K >= BKB && K % BKB == 0; }

hipError_t int8_mm(const int8_t* A, const float* sa, const int8_t* B, const float* sb, const float* addend,
                   const void* bias, int bias_dtype, int M, int N, int K, void* y, int y_dtype, hipStream_t s) {
  if (M <= 0 || N <= 0) return hipSuccess;
  if (K % 16 != 0) return hipErrorInvalidValue;
  const I8Epi e{sa, sb, addend, bias, bias_dtype, y, y_dtype, M, N};
  const bool aligned = (reinterpret_cast<uintptr_t>(A) & 15) == 0 && (reinterpret_cast<uintptr_t>(B) & 15) == 0;
  if (aligned && int8_mm_tiled_supported(M, N, K)) {
    const int tm2 = (M + TB - 1) / TB, tn2 = (N + TB - 1) / TB;
    if (tm2 * tn2 >= 256) {  // enough 256x256 tiles to fill the 256 CUs once
      static bool attr = false;
      if (!attr) {
        PTDT_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&i8_mm_t256_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, TB_LDS));
        attr = true;
      }
      hipLaunchKernelGGL(i8_mm_t256_kernel, dim3(tm2 * tn2), dim3(512), TB_LDS, s, A, B, K, e, tm2, tn2);
      return hipGetLastError();
    }
    const int tm = (M + TM - 1) / TM, tn = (N + TN - 1) / TN;
    hipLaunchKernelGGL(i8_mm_tiled_kernel, dim3(tm * tn), dim3(kThreads), LDS_BYTES, s, A, B, K, e, tm, tn);
    return hipGetLastError();
  }
  const int tm = (M + 63) / 64, tn = (N + 63) / 64;
  hipLaunchKernelGGL(i8_mm_kernel, dim3(tm * tn), dim3(kThreads), 0, s, A, B, K, e, tm, tn);
  return hipGetLastError();
}

}  // namespace ptdt
