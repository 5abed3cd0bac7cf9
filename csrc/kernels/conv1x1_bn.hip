// Streaming 1x1 convolution + BatchNorm batch statistics for the memory-bound ResNet shapes
// (ops/convbn.py; the tiled gemm_bn_stats in gemm_big.hip covers the rest).
//
//   Y[M, N] = X[M, K] . W[N, K]^T  (bf16 in/out, fp32 MFMA accumulate), M = N*H*W rows of an NHWC
//   activation, and per output channel c: sum(Y - P_c), sum((Y - P_c)^2) over the stored bf16 Y,
//   P_c = the BN's running_mean (a pivot close to the batch mean: the merge is plain summation and
//   E[(y-P)^2] - E[y-P]^2 does not cancel), merged into mean / invstd / scale / shift + running stats.
//
// Why a second kernel: at K = 64..256 and N = 64..256 the GEMM is pure streaming (layer1 of
// ResNet-50 at batch 128: 51-205 MB in, 51-205 MB out per conv, ~1 FLOP per byte), and a
// one-tile-per-workgroup GEMM serialises load -> MFMA -> LDS-staged epilogue inside every
// workgroup: 113-127 us for 64 -> 256 channels vs MIOpen's 42 (profiles/r3_convbn.md). Here:
//   * persistent workgroups (2 per CU), W resident in LDS for the whole launch (N*K*2 <= 64 KiB),
//     loaded once and stored in the MFMA-row order below;
//   * X row blocks of 16*NW rows LDS-DMA'd (global_load_lds_dwordx4) NBUF = 3 deep: block t+2 is
//     in flight while block t is multiplied and stored, waits are counted vmcnt (the DMAs and
//     the stores of the two previous blocks stay in flight);
//   * MFMA with W as the A operand: D[n][m] = sum_k W[n][k] X[m][k]; lane (fr, fq) of a 16x16
//     result holds rows n = 4fq..4fq+3 of column m = fr. W's rows are laid out so that col-frags
//     2p and 2p+1 cover channels 32p + 8fq + {0..3} and 32p + 8fq + {4..7}: each lane then owns 8
//     consecutive channels of one output row per pair -> one 16-B global store, no LDS epilogue;
//   * statistics accumulate per lane in registers over the whole launch (its rows, its N/4
//     channels), are reduced once at the end (DPP within the 16 lanes of a row, LDS across
//     waves) into one [2, N] partial per workgroup, and merged by the last workgroup of each
//     group / the last group (sc1 stores and loads + ticket, as gemm_bn_stats).
#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;
typedef __attribute__((address_space(1))) float gfloat;

__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store((gfloat*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load((gfloat*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

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

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// workgroup barrier without __syncthreads' fence (which would drain every in-flight DMA and store):
// LDS traffic retired, then s_barrier
__device__ __forceinline__ void bar() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// 16-B chunk c of LDS row r (rows of K bf16) is stored in slot swz(r, c) of the row, so the 16 lanes of
// a fragment read (16 consecutive rows, one chunk) hit 16 distinct 16-B slots
template <int K>
__device__ __forceinline__ int swz(int r, int c) {
  // rows of 128 B (K = 64): XOR the 8 chunks of the row by (r >> 1) & 7 (two rows share a 256-B bank row);
  // rows of >= 256 B: XOR the chunk index by r & 15, so 16 consecutive rows land on 16 distinct 16-B slots
  // of the bank row (the (r >> 1) & 7 form left two rows of a fragment read on one bank: PMC
  // SQ_LDS_BANK_CONFLICT 3.6-7.2M cycles per launch, profiles/r3_pmc_convbn_stream.md). An involution.
  if constexpr (K >= 128) return c ^ (r & 15);
  else return (c & ~7) | ((c & 7) ^ ((r >> 1) & 7));
}
template <int K>
__device__ __forceinline__ int lds_off(int r, int c) {
  return r * (K * 2) + swz<K>(r, c) * 16;
}

// compile-time loop: f(std::integral_constant<int, i>) for i = 0 .. n-1
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// lane (I % 16) of this lane's 16-lane DPP row, register I / 16 (row_newbcast)
template <int I, int R>
__device__ __forceinline__ float row_bcast(const float (&r)[R]) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, r[I >> 4]),
                                                               0x150 + (I & 15), 0xF, 0xF, false));
}

template <int K, int N, int NW, int NB, int NS>
struct C1 {
  static constexpr int NT = NW * 64;
  static constexpr int BM = 16 * NW;         // rows per block (16 per wave)
  static constexpr int NSL = N / NS;         // channels of one weight slab (one workgroup's share)
  static constexpr int WB = NSL * K * 2;     // resident weights
  static constexpr int AB = BM * K * 2;      // one X block
  // X blocks in flight + 1: NB, or fewer where the LDS does not hold them
  static constexpr int NBUF = WB + NB * AB <= 160 * 1024 ? NB : (WB + 3 * AB <= 160 * 1024 ? 3 : 2);
  // workgroups per CU: two waves per SIMD (the register budget), and the LDS
  static constexpr int PER_CU = (8 / NW) * (WB + NBUF * AB) <= 160 * 1024 ? 8 / NW : 1;
  static constexpr int DMA = AB / (NT * 16); // LDS-DMAs per thread per block
  static constexpr int NP = NSL / 32;        // channel pairs (2 col-frags, 32 channels)
  static constexpr int KS = K / 32;          // MFMA k-steps
  static constexpr int LDS = WB + NBUF * AB;
  static constexpr int CH = NSL < 128 ? NSL : 128;  // channels per chunk of the MFMA/epilogue loop
  static constexpr int CP = CH / 32;            // pairs per chunk
  static constexpr int PR = (8 * NP + 15) / 16; // pivot registers per lane (see below)
  static_assert(AB % (NT * 16) == 0 && NSL % 32 == 0 && N % NS == 0 && K % 64 == 0, "shape");
  static constexpr bool FITS = LDS <= 160 * 1024;  // dispatch() only launches configurations that fit
  static_assert(2 * NW * NSL * 4 + 16 <= NBUF * AB, "cross-wave statistics scratch");
};

// weight row of col-frag j's MFMA row fr (see the header): channel 32p + 8(fr/4) + 4(j%2) + fr%4
__device__ __forceinline__ int w_channel(int j, int fr) { return 32 * (j >> 1) + 8 * (fr >> 2) + 4 * (j & 1) + (fr & 3); }

template <int K, int N, int NW, int NB, int NS>
__global__ void __launch_bounds__(NW * 64, 2) conv1x1_bn_stream_kernel(const uint16_t* __restrict__ X,
                                                                       const uint16_t* __restrict__ W,
                                                                       uint16_t* __restrict__ Y, int M,
                                                                       GemmBnEpi e, int nblk) {
  using S = C1<K, N, NW, NB, NS>;
  static_assert(S::FITS, "LDS");
  constexpr int NSL = S::NSL;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* wl = smem;
  uint8_t* al = smem + S::WB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  // workgroup = (row workgroup rwg, weight slab): NS workgroups share each row block, one per slab
  // of NSL output channels (X is read NS times; the repeats mostly hit the 256 MiB Infinity Cache)
  const int slab = (int)blockIdx.x % NS, rwg = (int)blockIdx.x / NS;
  const int G = (int)gridDim.x / NS;  // row workgroups
  const int n0 = slab * NSL;

  // X block t of this workgroup: rows (blockIdx.x + t*G) * BM ..; rows past M clamp to M-1 (computed,
  // never stored, not counted)
  auto stage = [&](int t) {
    const int blk = rwg + t * G;
    const int row0 = blk * S::BM;
    uint8_t* dst0 = al + (t % S::NBUF) * S::AB;
#pragma unroll
    for (int i = 0; i < S::DMA; ++i) {
      const int p = i * S::NT + tid;  // 16-B chunk of the block image (linear LDS order)
      const int r = p / (K / 8), slot = p % (K / 8);
      // the chunk stored in LDS slot `slot` of row r is logical chunk c (the swizzle is an involution)
      const int c = swz<K>(r, slot);
      const int gr = min(row0 + r, M - 1);
      const uint16_t* g = X + (int64_t)gr * K + c * 8;
      __builtin_amdgcn_global_load_lds((gbl_void*)g, (lds_void*)(dst0 + (i * S::NT + wid * 64) * 16), 16, 0, 0);
    }
  };
  const int nt = (nblk - rwg + G - 1) / G;  // blocks of this workgroup (>= 1: row workgroups <= nblk)

#pragma unroll
  for (int t = 0; t < S::NBUF - 1; ++t)
    if (t < nt) stage(t);
  // resident weights in MFMA row order (plain loads + LDS stores, once)
  for (int p = tid; p < NSL * (K / 8); p += S::NT) {
    const int r = p / (K / 8), c = p % (K / 8);  // LDS row r = (col-frag j, MFMA row fr)
    const int ch = n0 + w_channel(r >> 4, r & 15);
    *reinterpret_cast<uint4*>(wl + lds_off<K>(r, c)) = *reinterpret_cast<const uint4*>(W + (int64_t)ch * K + c * 8);
  }
  // pivots (the running mean, or 0) for the lane's channels 32p + 8fq + q, spread over the 16 lanes of
  // its DPP row: value i = 8p + q sits in register i / 16 of lane fr = i % 16 and is broadcast with
  // row_newbcast when used (pivots read from LDS inside the loop would make the compiler drain every
  // in-flight LDS-DMA and store first; 8*NP registers per lane would not fit beside the sums)
  float pivr[S::PR];
#pragma unroll
  for (int k = 0; k < S::PR; ++k) {
    const int i = 16 * k + fr;
    pivr[k] = (e.p.running_mean && i < 8 * S::NP) ? e.p.running_mean[n0 + 32 * (i >> 3) + 8 * fq + (i & 7)] : 0.f;
  }
  // drain the prologue (the first X blocks, weights): from here on the counted waits are exact
  vm_wait<0>();
  float s1[S::NP][8], s2[S::NP][8];
#pragma unroll
  for (int p = 0; p < S::NP; ++p)
#pragma unroll
    for (int v = 0; v < 8; ++v) s1[p][v] = s2[p][v] = 0.f;

  constexpr int D = S::NBUF - 1;  // blocks in flight ahead of the one being multiplied
  for (int t = 0; t < nt; ++t) {
    bar();  // block t-1's buffer ((t+D) % NBUF) fully read; weights written (t = 0)
    if (t + D < nt) stage(t + D);
    // retire block t: issued after its DMAs are the stores of blocks t-D .. t-1 (NP each per thread)
    // and the DMAs of the blocks t+1 .. t+D that exist (blocks < D were drained in the prologue)
    const int ahead = min(D, nt - 1 - t);
    static_for<0, D + 1>([&](auto ac) {
      if (ahead == decltype(ac)::value) vm_wait<D * S::NP + decltype(ac)::value * S::DMA>();
    });
    bar();  // every wave's part of block t is in LDS
    const uint8_t* at = al + (t % S::NBUF) * S::AB;
    bf16x8_t xb[S::KS];
#pragma unroll
    for (int ks = 0; ks < S::KS; ++ks)
      xb[ks] = *reinterpret_cast<const bf16x8_t*>(at + lds_off<K>(wid * 16 + fr, ks * 4 + fq));
    const int m = (rwg + t * G) * S::BM + wid * 16 + fr;
    const bool valid = m < M;
    // a row past M multiplied the clamped row M-1: it stores row M-1's identical bytes there, so
    // every wave issues the same store count (the counted waits) and no lane diverges
    const int64_t ms = valid ? m : M - 1;
    static_for<0, NSL / S::CH>([&](auto chc) {  // channel chunks: 2*CP accumulator tiles live at a time
      constexpr int ch = decltype(chc)::value;
      f32x4_t acc[2 * S::CP];
#pragma unroll
      for (int j = 0; j < 2 * S::CP; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < S::KS; ++ks)
#pragma unroll
        for (int j = 0; j < 2 * S::CP; ++j) {
          const int jj = ch * 2 * S::CP + j;
          const bf16x8_t wa = *reinterpret_cast<const bf16x8_t*>(wl + lds_off<K>(jj * 16 + fr, ks * 4 + fq));
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, xb[ks], acc[j], 0, 0, 0);
        }
      static_for<0, S::CP>([&](auto ppc) {
        constexpr int pp = decltype(ppc)::value;
        constexpr int p = ch * S::CP + pp;
        uint32_t h2[4];  // bf16 pairs: v_cvt_pk_bf16_f32 (gfx950, round to nearest even)
        static_for<0, 4>([&](auto qc) {
          constexpr int q2 = decltype(qc)::value;
          const auto& a = acc[2 * pp + (q2 >> 1)];
          const f32x2_t f = {a[(2 * q2) & 3], a[(2 * q2 + 1) & 3]};
          h2[q2] = __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2_t));
        });
        static_for<0, 8>([&](auto qc) {
          constexpr int q = decltype(qc)::value;
          const float y = __uint_as_float((q & 1) ? (h2[q >> 1] & 0xffff0000u) : (h2[q >> 1] << 16));
          // pivot of channel 32p + 8fq + q: value 8p + q of the row (see the prologue). Broadcast by
          // every lane, outside the `valid` select: a DPP read from a lane masked off in EXEC returns 0
          const float piv = row_bcast<8 * p + q>(pivr);
          const float d = valid ? y - piv : 0.f;
          s1[p][q] += d;
          s2[p][q] = fmaf(d, d, s2[p][q]);
        });
        uint4 u;
        u.x = h2[0];
        u.y = h2[1];
        u.z = h2[2];
        u.w = h2[3];
        *reinterpret_cast<uint4*>(Y + ms * N + n0 + 32 * p + 8 * fq) = u;
      });
    });
  }

  // reduce the lane statistics: over the 16 lanes of a DPP row (rows of the block), then the waves
#pragma unroll
  for (int p = 0; p < S::NP; ++p)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float a = s1[p][q], b = s2[p][q];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        a += __shfl_xor(a, o);
        b += __shfl_xor(b, o);
      }
      s1[p][q] = a;
      s2[p][q] = b;
    }
  __syncthreads();  // the X buffers are free: reuse them for the cross-wave sums
  float* red = reinterpret_cast<float*>(al);  // [NW][2][N]
  if (fr == 0) {
#pragma unroll
    for (int p = 0; p < S::NP; ++p)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        red[(wid * 2 + 0) * NSL + 32 * p + 8 * fq + q] = s1[p][q];
        red[(wid * 2 + 1) * NSL + 32 * p + 8 * fq + q] = s2[p][q];
      }
  }
  __syncthreads();
  float* ws1 = e.ws;
  float* ws2 = e.ws + (int64_t)G * N;
  for (int c = tid; c < NSL; c += S::NT) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      a += red[(w * 2 + 0) * NSL + c];
      b += red[(w * 2 + 1) * NSL + c];
    }
    st_sc1(ws1 + (int64_t)rwg * N + n0 + c, a);
    st_sc1(ws2 + (int64_t)rwg * N + n0 + c, b);
  }

  // two-level merge (fixed order: deterministic)
  int* flag = reinterpret_cast<int*>(red + 2 * NW * NSL);
  const int GS = e.group, ng = (G + GS - 1) / GS;
  const int gi = rwg / GS, g0 = gi * GS, gc = min(GS, G - g0);
  int* tk = e.tickets + slab * (ng + 1);  // this slab's group tickets, then its final ticket
  if (!last_arrival(tk + gi, gc, flag)) return;
  float* gs1 = e.ws + (int64_t)2 * G * N;
  float* gs2 = gs1 + (int64_t)ng * N;
  for (int cc = tid; cc < NSL; cc += S::NT) {
    const int c = n0 + cc;
    double a = 0.0, b = 0.0;
    for (int k = g0; k < g0 + gc; ++k) {
      a += (double)ld_sc1(ws1 + (int64_t)k * N + c);
      b += (double)ld_sc1(ws2 + (int64_t)k * N + c);
    }
    st_sc1(gs1 + (int64_t)gi * N + c, (float)a);
    st_sc1(gs2 + (int64_t)gi * N + c, (float)b);
  }
  if (!last_arrival(tk + ng, ng, flag)) return;
  const BnParams& bp = e.p;
  const double Md = (double)M;
  for (int cc = tid; cc < NSL; cc += S::NT) {
    const int c = n0 + cc;
    double a = 0.0, b = 0.0;
    for (int k = 0; k < ng; ++k) {
      a += (double)ld_sc1(gs1 + (int64_t)k * N + c);
      b += (double)ld_sc1(gs2 + (int64_t)k * N + c);
    }
    const double ms = a / Md;
    double var = b / Md - ms * ms;
    if (var < 0.0) var = 0.0;
    const double mean = (bp.running_mean ? (double)bp.running_mean[c] : 0.0) + ms;
    const float invstd = (float)(1.0 / sqrt(var + (double)bp.eps));
    const float w = bp.weight ? bp.weight[c] : 1.f, bb = bp.bias ? bp.bias[c] : 0.f;
    bp.mean[c] = (float)mean;
    bp.invstd[c] = invstd;
    bp.scale[c] = w * invstd;
    bp.shift[c] = bb - (float)mean * w * invstd;
    if (bp.running_mean) {
      const double unbiased = M > 1 ? var * Md / (Md - 1.0) : var;
      bp.running_mean[c] = (float)((1.0 - bp.momentum) * bp.running_mean[c] + bp.momentum * mean);
      bp.running_var[c] = (float)((1.0 - bp.momentum) * bp.running_var[c] + bp.momentum * unbiased);
    }
  }
  if (tid == 0 && slab == 0 && bp.num_batches_tracked) *bp.num_batches_tracked += 1;
}

constexpr int kCus = 256;

int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return (v && v[0]) ? atoi(v) : dflt;
}

int stream_group(int G) {
  int g = 1;
  while (g * g < G) ++g;
  return g;
}

// row workgroups (the grid is that times NS): enough to hold PER_CU workgroups on every CU
template <class S, int NS>
int rows_of(int M) {
  const int nblk = (M + S::BM - 1) / S::BM;
  int g = kCus * S::PER_CU / NS;
  if (g < 1) g = 1;
  return nblk < g ? nblk : g;
}

template <int K, int N, int NW, int NB, int NS>
hipError_t launch_stream(const void* X, const void* W, void* Y, int M, GemmBnEpi e, hipStream_t s) {
  using S = C1<K, N, NW, NB, NS>;
  const void* fn = reinterpret_cast<const void*>(&conv1x1_bn_stream_kernel<K, N, NW, NB, NS>);
  static bool attr_set = false;
  if (!attr_set) {
    PTDT_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, S::LDS));
    attr_set = true;
  }
  const int G = rows_of<S, NS>(M);
  e.group = stream_group(G);
  hipLaunchKernelGGL((conv1x1_bn_stream_kernel<K, N, NW, NB, NS>), dim3(G * NS), dim3(S::NT), S::LDS, s,
                     static_cast<const uint16_t*>(X), static_cast<const uint16_t*>(W), static_cast<uint16_t*>(Y), M,
                     e, (M + S::BM - 1) / S::BM);
  return hipGetLastError();
}

// pipeline configurations (waves per workgroup, X buffers): 0 = (4, 3), 1 = (4, 5), 2 = (8, 2), 3 = (8, 3).
// PTDT_C1_CFG overrides the per-shape default (benchmarks/conv1x1_fwd_probe.py --sweep).
int cfg_for(int K, int N) {
  const int forced = env_int("PTDT_C1_CFG", -1);  // read per call: benchmarks sweep it in one process
  if (forced >= 0 && forced <= 3) return forced;
  // measured (profiles/r3_convbn_stream_sweep*.jsonl): 8 waves x 2 buffers for K = 64 (31.3 vs 35.1 us
  // at 64 -> 64, 65.0 vs 69.2 at 64 -> 256) and 128 -> 512 (47.1 vs 48.5); within noise for K = 256
  (void)N;
  return K <= 128 ? 2 : 0;
}

// (K, N, weight slabs) instances: ResNet-50's stride-1 1x1 convolutions whose weights fit the LDS
// whole (layer1) or in NS slabs of <= 64 KiB
template <class F>
bool dispatch(int K, int N, F&& f) {
  const int cfg = cfg_for(K, N);
  auto go = [&](auto k, auto n, auto ns) {
    auto run = [&](auto nw, auto nb) {
      constexpr int kk = decltype(k)::value, nn = decltype(n)::value, s_ = decltype(ns)::value;
      if constexpr (C1<kk, nn, decltype(nw)::value, decltype(nb)::value, s_>::FITS) f(k, n, nw, nb, ns);
      else f(k, n, std::integral_constant<int, 4>{}, std::integral_constant<int, 3>{}, ns);
    };
    switch (cfg) {
      case 1: run(std::integral_constant<int, 4>{}, std::integral_constant<int, 5>{}); break;
      case 2: run(std::integral_constant<int, 8>{}, std::integral_constant<int, 2>{}); break;
      case 3: run(std::integral_constant<int, 8>{}, std::integral_constant<int, 3>{}); break;
      default: run(std::integral_constant<int, 4>{}, std::integral_constant<int, 3>{}); break;
    }
  };
#define PTDT_C1(k, n, ns)                                                                                  \
  if (K == k && N == n) {                                                                                \
    go(std::integral_constant<int, k>{}, std::integral_constant<int, n>{}, std::integral_constant<int, ns>{}); \
    return true;                                                                                         \
  }
  // 64 -> 256 as two 128-channel slabs: half the per-lane statistics registers (152 VGPRs, 3 waves per
  // SIMD instead of 2), X read twice: 60.3 vs 65.8 us (profiles/r3_convbn_stream_sweep_split.jsonl);
  // PTDT_C1_SPLIT=0 keeps one slab
  if (K == 64 && N == 256 && env_int("PTDT_C1_SPLIT", 1) == 1) {
    go(std::integral_constant<int, 64>{}, std::integral_constant<int, 256>{}, std::integral_constant<int, 2>{});
    return true;
  }
  PTDT_C1(64, 64, 1) PTDT_C1(64, 256, 1) PTDT_C1(256, 64, 1) PTDT_C1(256, 128, 1)
  PTDT_C1(128, 512, 4) PTDT_C1(256, 1024, 8)
#undef PTDT_C1
  return false;
}

}  // namespace

bool conv1x1_bn_stream_supported(int K, int N) {
  return dispatch(K, N, [](auto, auto, auto, auto, auto) {});
}

// (row workgroups, weight slabs) of the launch for this shape
static void stream_geometry(int M, int K, int N, int* G, int* NS) {
  *G = 0, *NS = 1;
  dispatch(K, N, [&](auto k, auto n, auto nw, auto nb, auto ns) {
    constexpr int s_ = decltype(ns)::value;
    *G = rows_of<C1<decltype(k)::value, decltype(n)::value, decltype(nw)::value, decltype(nb)::value, s_>, s_>(M);
    *NS = s_;
  });
}

int64_t conv1x1_bn_stream_ws_floats(int M, int K, int N) {
  int G, NS;
  stream_geometry(M, K, N, &G, &NS);
  const int ng = (G + stream_group(G) - 1) / stream_group(G);
  return (int64_t)2 * N * (G + ng);
}

int conv1x1_bn_stream_num_tickets(int M, int K, int N) {
  int G, NS;
  stream_geometry(M, K, N, &G, &NS);
  return NS * ((G + stream_group(G) - 1) / stream_group(G) + 1);
}

hipError_t conv1x1_bn_stream(const void* X, const void* W, void* Y, int M, int K, int N, GemmBnEpi e,
                             hipStream_t s) {
  if (M <= 0 || e.ws == nullptr || e.tickets == nullptr || e.p.mean == nullptr || e.p.scale == nullptr)
    return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(W) | reinterpret_cast<uintptr_t>(Y)) & 15)
    return hipErrorInvalidValue;
  hipError_t err = hipErrorInvalidValue;
  dispatch(K, N, [&](auto k, auto n, auto nw, auto nb, auto ns) {
    err = launch_stream<decltype(k)::value, decltype(n)::value, decltype(nw)::value, decltype(nb)::value,
                        decltype(ns)::value>(X, W, Y, M, e, s);
  });
  return err;
}

}  // namespace ptdt
