// Backward of ``BN(conv1x1(X))`` for the streaming ResNet shapes (ops/convbn.py), fused:
//
//   dY[m, n] = A[n] g[m, n] + B[n] y[m, n] + C[n]      (the BN backward's apply, never stored)
//   dX[M, K] = dY . W                                  (data gradient, bf16 out)
//   dW[N, K] = dY^T . X                                (weight gradient, fixed-order merge, bf16 out)
//
// g is the BN's masked incoming gradient (ReLU mask applied, residual link added) written by the BN
// backward's reduce pass, y the conv output (the BN input), A/B/C the per-channel coefficients that
// pass computes (batchnorm.hip). Unfused, the apply pass reads g and y and writes dY, MIOpen's data
// gradient reads dY, its weight gradient reads dY and X and zero-fills / casts around its atomic
// accumulation (profiles/r3_resnet_step_breakdown.md: 1.2 ms of helpers per step). Here every row
// block of g, y and X is read once.
//
// Per workgroup (4 waves, persistent over row blocks of BM = 64):
//   * W^T resident in LDS ([K][N], padded rows) for the data gradient's A operand, rows permuted so a
//     lane's two tiles of a pair cover 8 consecutive input channels (one 16-B dX store);
//   * each wave computes dY for its 16 rows straight from 16-B loads of g and y (the data gradient's
//     B operand as it stands) and writes it to a padded LDS image; X's 64 rows go to another;
//   * weight gradient: both operands are column slices of those row-major images, read with
//     ds_read_b64_tr_b16 (gfx950's transposing LDS read); fp32 accumulators per wave for the whole
//     launch (N*K/256 values per lane);
//   * partials [workgroup][N][K] (plain stores) summed by a second kernel in a fixed order:
//     deterministic. (The first version merged in-kernel -- last arrival of each group, sc1 loads one
//     partial at a time: ~800 us per call at layer1's 512 partials of 64 KB; ResNet-50 step 20.2 vs
//     16.3 ms unfused, profiles/r4_resnet_step.md.)
#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;  // native vector: register arrays of it stay in VGPRs
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4;
typedef __attribute__((address_space(1))) float gfloat;

constexpr int kBwdWaves = 4;
constexpr int kBwdThreads = 64 * kBwdWaves;
constexpr int kBwdBM = 64;  // rows per block (16 per wave for the data gradient)

// input channel of row i of data-gradient A tile j (a pair of tiles covers 32 channels; lane group q
// of the pair holds channels 32p + 8q .. +7)
__device__ __forceinline__ int k_of(int j, int i) { return 32 * (j >> 1) + 8 * (i >> 2) + 4 * (j & 1) + (i & 3); }

template <int K, int N>
struct Cb {
  static constexpr int SWT = 2 * N + 16;  // W^T row stride (bytes): 16-B chunk reads spread over banks
  static constexpr int SDY = 2 * N + 16;  // dY image rows
  static constexpr int SX = 2 * K + 16;   // X image rows
  static constexpr int WT_B = K * SWT;
  static constexpr int DY_B = kBwdBM * SDY;
  static constexpr int X_B = kBwdBM * SX;
  static constexpr int CO_B = 3 * N * 4;  // A, B, C coefficients
  static constexpr int LDS = WT_B + DY_B + X_B + CO_B;
  static constexpr int PER_CU = 2 * LDS <= 160 * 1024 ? 2 : 1;
  static constexpr int NS = N / 32;        // k-steps of the data gradient (over N)
  static constexpr int KP = K / 32;        // output channel pairs of the data gradient
  static constexpr int NTW = N / 64;       // weight-gradient n-tiles per wave
  static constexpr int KT = K / 16;        // weight-gradient k-tiles
  static constexpr int XCH = K / 8;        // 16-B chunks per X row
  static constexpr int XPL = 16 * XCH / 64;  // X chunks per lane (a wave stages its 16 rows)
  static_assert(N % 64 == 0 && K % 32 == 0 && (16 * XCH) % 64 == 0, "shape");
  static_assert(LDS <= 160 * 1024, "LDS");
};

template <int K, int N>
__global__ void __launch_bounds__(kBwdThreads, 2) conv1x1_bwd_kernel(
    const uint16_t* __restrict__ G, const uint16_t* __restrict__ Y, const uint16_t* __restrict__ X,
    const uint16_t* __restrict__ W, const float* __restrict__ coef, uint16_t* __restrict__ dX,
    float* __restrict__ ws, int M, int nblk) {
  using S = Cb<K, N>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* const wt = smem;
  uint8_t* const dyi = wt + S::WT_B;
  uint8_t* const xi = dyi + S::DY_B;
  float* const co = reinterpret_cast<float*>(xi + S::X_B);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int rwg = blockIdx.x, Gn = gridDim.x;

  // ---- prologue: W^T (permuted rows) and the coefficients into LDS
  for (int e = tid; e < N * (K / 8); e += kBwdThreads) {
    const int n = e / (K / 8), kc = e % (K / 8);
    const u32x4_t v = *reinterpret_cast<const u32x4_t*>(W + (int64_t)n * K + kc * 8);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = kc * 8 + u;
      // LDS row r of tile j holds channel k_of(j, i): r = 16 j + i with k_of(j, i) = k
      const int j = 2 * (k >> 5) + ((k >> 2) & 1), i = 4 * ((k >> 3) & 3) + (k & 3);
      *reinterpret_cast<uint16_t*>(wt + (16 * j + i) * S::SWT + n * 2) = (uint16_t)(v[u >> 1] >> (16 * (u & 1)));
    }
  }
  for (int e = tid; e < 3 * N; e += kBwdThreads) co[e] = coef[e];

  f32x4_t wacc[S::NTW][S::KT];
#pragma unroll
  for (int a = 0; a < S::NTW; ++a)
#pragma unroll
    for (int t = 0; t < S::KT; ++t) wacc[a][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  __syncthreads();

  for (int blk = rwg; blk < nblk; blk += Gn) {
    const int m0 = blk * kBwdBM;
    // ---- loads: this wave's 16 rows of g and y (row fr, channels 32 s + 8 fq ..), and of X
    const int mr = m0 + 16 * w + fr;
    const bool valid = mr < M;
    const int64_t mc = valid ? mr : M - 1;
    u32x4_t gv[S::NS], yv[S::NS], xv[S::XPL];
#pragma unroll
    for (int s = 0; s < S::NS; ++s) {
      gv[s] = *reinterpret_cast<const u32x4_t*>(G + mc * N + 32 * s + 8 * fq);
      yv[s] = *reinterpret_cast<const u32x4_t*>(Y + mc * N + 32 * s + 8 * fq);
    }
#pragma unroll
    for (int u = 0; u < S::XPL; ++u) {
      const int e = lane + 64 * u, r = e / S::XCH, c = e % S::XCH;
      const int xr = m0 + 16 * w + r;
      xv[u] = *reinterpret_cast<const u32x4_t*>(X + (int64_t)(xr < M ? xr : M - 1) * K + c * 8);
    }
    __syncthreads();  // the previous block's weight-gradient reads of the images are done
#pragma unroll
    for (int u = 0; u < S::XPL; ++u) {
      const int e = lane + 64 * u, r = e / S::XCH, c = e % S::XCH;
      *reinterpret_cast<u32x4_t*>(xi + (16 * w + r) * S::SX + c * 16) = xv[u];
    }
    // ---- dY (bf16) for the data gradient's B operand and the image
    bf16x8_t dyb[S::NS];
#pragma unroll
    for (int s = 0; s < S::NS; ++s) {
      const int n0 = 32 * s + 8 * fq;
      const f32x4_t* ca = reinterpret_cast<const f32x4_t*>(co + n0);
      const f32x4_t* cb = reinterpret_cast<const f32x4_t*>(co + N + n0);
      const f32x4_t* cc = reinterpret_cast<const f32x4_t*>(co + 2 * N + n0);
      float d[8];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4_t A4 = ca[h], B4 = cb[h], C4 = cc[h];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e = 4 * h + u;
          const float gg = bf16_to_f32((uint16_t)(gv[s][e >> 1] >> (16 * (e & 1))));
          const float yy = bf16_to_f32((uint16_t)(yv[s][e >> 1] >> (16 * (e & 1))));
          d[4 * h + u] = valid ? fmaf(A4[u], gg, fmaf(B4[u], yy, C4[u])) : 0.f;
        }
      }
      u32x4_t pk;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const f32x2_t f = {d[2 * h], d[2 * h + 1]};
        pk[h] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2_t));
      }
      dyb[s] = __builtin_bit_cast(bf16x8_t, pk);
      *reinterpret_cast<u32x4_t*>(dyi + (16 * w + fr) * S::SDY + n0 * 2) = pk;
    }
    // ---- data gradient: dX[m][k] = sum_n W^T[k][n] dY[m][n], two tiles (32 channels) at a time
#pragma unroll
    for (int p = 0; p < S::KP; ++p) {
      f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int s = 0; s < S::NS; ++s)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const bf16x8_t a =
              *reinterpret_cast<const bf16x8_t*>(wt + (16 * (2 * p + h) + fr) * S::SWT + (32 * s + 8 * fq) * 2);
          acc[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, dyb[s], acc[h], 0, 0, 0);
        }
      if (valid) {
        u32x4_t pk;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const f32x4_t& a = acc[h >> 1];
          const f32x2_t f = {a[(2 * h) & 3], a[(2 * h + 1) & 3]};
          pk[h] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2_t));
        }
        *reinterpret_cast<u32x4_t*>(dX + (int64_t)mr * K + 32 * p + 8 * fq) = pk;
      }
    }
    __syncthreads();  // both images complete
    // ---- weight gradient: dW[n][k] += sum_m dY[m][n] X[m][k] over this block's 64 rows; A = dY^T and
    // B = X^T are column slices of the row-major images: ds_read_b64_tr_b16 (lane 4q+p of a 16-lane
    // group addresses row q, columns 4p..4p+3 of a 4 x 16 block; lane i receives column i)
    const int tq = fr >> 2, tp = fr & 3;
#pragma unroll
    for (int ks = 0; ks < kBwdBM / 32; ++ks) {
      const int rb = 32 * ks + 8 * fq + tq;  // block row of this lane's address (first read; +4 second)
      bf16x8_t af[S::NTW], bfv[S::KT];
#pragma unroll
      for (int a = 0; a < S::NTW; ++a) {
        const int n0 = (w * S::NTW + a) * 16 + 4 * tp;
        const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(dyi + rb * S::SDY + n0 * 2));
        const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(dyi + (rb + 4) * S::SDY + n0 * 2));
        af[a] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int t = 0; t < S::KT; ++t) {
        const int k0 = t * 16 + 4 * tp;
        const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xi + rb * S::SX + k0 * 2));
        const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(xi + (rb + 4) * S::SX + k0 * 2));
        bfv[t] = __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int a = 0; a < S::NTW; ++a)
#pragma unroll
        for (int t = 0; t < S::KT; ++t)
          wacc[a][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bfv[t], wacc[a][t], 0, 0, 0);
    }
  }

  // ---- weight-gradient partial of this workgroup (lane (fr, fq) of tile (a, t): dW[n = 16 nt + 4 fq + r][k = 16 t + fr])
  float* const wp = ws + (int64_t)rwg * N * K;
#pragma unroll
  for (int a = 0; a < S::NTW; ++a)
#pragma unroll
    for (int t = 0; t < S::KT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) wp[(int64_t)((w * S::NTW + a) * 16 + 4 * fq + r) * K + 16 * t + fr] = wacc[a][t][r];
}

// dW = sum of the G partials [G][NK] in a fixed order: 16 waves per workgroup, each 64 float4
// columns; wave v sums partials v, v + 16, ... (4 loads in flight per lane), the 16 wave sums meet
// in LDS and wave 0 adds them in wave order. The kernel boundary makes the partials visible.
constexpr int kMergeWaves = 16;
__global__ void __launch_bounds__(64 * kMergeWaves) conv1x1_bwd_merge_kernel(const float* __restrict__ ws, int G,
                                                                             int nk4, uint16_t* __restrict__ dW) {
  __shared__ f32x4_t part[kMergeWaves][64];
  const int lane = threadIdx.x & 63, v = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;  // float4 column
  const f32x4_t* const src = reinterpret_cast<const f32x4_t*>(ws);
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  if (c < nk4) {
    int q = v;
    for (; q + 3 * kMergeWaves < G; q += 4 * kMergeWaves) {
      const f32x4_t a0 = src[(int64_t)q * nk4 + c], a1 = src[(int64_t)(q + kMergeWaves) * nk4 + c];
      const f32x4_t a2 = src[(int64_t)(q + 2 * kMergeWaves) * nk4 + c], a3 = src[(int64_t)(q + 3 * kMergeWaves) * nk4 + c];
      acc += a0;
      acc += a1;
      acc += a2;
      acc += a3;
    }
    for (; q < G; q += kMergeWaves) acc += src[(int64_t)q * nk4 + c];
  }
  part[v][lane] = acc;
  __syncthreads();
  if (v != 0 || c >= nk4) return;
  f32x4_t sum = part[0][lane];
#pragma unroll
  for (int u = 1; u < kMergeWaves; ++u) sum += part[u][lane];
  uint2 pk;
  pk.x = (uint32_t)f32_to_bf16(sum[0]) | ((uint32_t)f32_to_bf16(sum[1]) << 16);
  pk.y = (uint32_t)f32_to_bf16(sum[2]) | ((uint32_t)f32_to_bf16(sum[3]) << 16);
  reinterpret_cast<uint2*>(dW)[c] = pk;
}

template <int K, int N>
int bwd_rows(int M) {
  const int nblk = (M + kBwdBM - 1) / kBwdBM;
  const int g = 256 * Cb<K, N>::PER_CU;
  return nblk < g ? nblk : g;
}

template <class F>
bool bwd_dispatch(int K, int N, F&& f) {
#define PTDT_C1B(k, n)                                                      \
  if (K == k && N == n) {                                                   \
    f(std::integral_constant<int, k>{}, std::integral_constant<int, n>{}); \
    return true;                                                            \
  }
  PTDT_C1B(64, 64) PTDT_C1B(64, 256) PTDT_C1B(256, 64) PTDT_C1B(256, 128)
#undef PTDT_C1B
  return false;
}

}  // namespace

bool conv1x1_bwd_supported(int K, int N) {
  return bwd_dispatch(K, N, [](auto, auto) {});
}

static void bwd_geometry(int M, int K, int N, int* G) {
  *G = 0;
  bwd_dispatch(K, N, [&](auto k, auto n) { *G = bwd_rows<decltype(k)::value, decltype(n)::value>(M); });
}

int64_t conv1x1_bwd_ws_floats(int M, int K, int N) {
  int G;
  bwd_geometry(M, K, N, &G);
  return (int64_t)G * N * K;
}

hipError_t conv1x1_bwd(const void* g, const void* y, const void* x, const void* w, const float* coef, void* dx,
                       void* dw, float* ws, int M, int K, int N, hipStream_t s) {
  if (M <= 0 || ws == nullptr) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(x) |
       reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(dx) | reinterpret_cast<uintptr_t>(dw) |
       reinterpret_cast<uintptr_t>(ws) | reinterpret_cast<uintptr_t>(coef)) & 15)
    return hipErrorInvalidValue;
  hipError_t err = hipErrorInvalidValue;
  int G = 0;
  bwd_dispatch(K, N, [&](auto k, auto n) {
    constexpr int kk = decltype(k)::value, nn = decltype(n)::value;
    using S = Cb<kk, nn>;
    const void* fn = reinterpret_cast<const void*>(&conv1x1_bwd_kernel<kk, nn>);
    static bool attr = false;
    if (!attr) {
      if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, S::LDS) != hipSuccess) return;
      attr = true;
    }
    G = bwd_rows<kk, nn>(M);
    hipLaunchKernelGGL((conv1x1_bwd_kernel<kk, nn>), dim3(G), dim3(kBwdThreads), S::LDS, s,
                       static_cast<const uint16_t*>(g), static_cast<const uint16_t*>(y),
                       static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(w), coef,
                       static_cast<uint16_t*>(dx), ws, M, (M + kBwdBM - 1) / kBwdBM);
    err = hipGetLastError();
  });
  if (err != hipSuccess) return err;
  const int nk4 = N * K / 4;
  hipLaunchKernelGGL(conv1x1_bwd_merge_kernel, dim3((nk4 + 63) / 64), dim3(64 * kMergeWaves), 0, s, ws, G, nk4,
                     static_cast<uint16_t*>(dw));
  return hipGetLastError();
}

}  // namespace ptdt
