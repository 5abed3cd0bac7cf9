// Fused DDP train step of a small Linear[-ReLU-Linear] model.
//
// Replaces, for the DDP toy workloads, the ~10 tiny ATen launches of the
// reference step (ddp_gpus.py:34-39: zero_grad, addmm, cross_entropy fwd,
// fill, cross_entropy bwd, addmm bwd, DDP bucket copy+scale, foreach SGD) plus
// its per-step H2D copies (ddp_gpus.py:47-48) with:
//   * an on-device gather of the batch from the resident dataset by sampler
//     indices (no DataLoader, no H2D per step),
//   * forward, loss, backward entirely in LDS,
//   * gradients written into the flat DDP bucket (the bucket IS the .grad
//     storage, no pack/unpack),
//   * the SGD update folded in: either the previous step's update applied
//     first from the already all-reduced bucket ("pre"), or -- with the
//     in-kernel one-shot xGMI all-reduce (csrc/comm/xgmi.h) -- this step's
//     update right after the all-reduce ("post"): one launch per DDP step.
// At these sizes (B=32, Din=20) the step is pure latency: one workgroup, all
// operands in LDS, no MFMA (a 32x1x20 product cannot fill a 16x16x32 tile).
//
// Two kernels share one step body:
//   fused_mlp_step_kernel       -- one DDP step per launch (hipGraph-captured),
//   fused_mlp_persistent_kernel -- n steps per launch. Measured on MI355X
//     (profiles/): a captured 1-workgroup kernel costs a 1.56 us node floor
//     plus ~1 us to re-read parameters that the previous step wrote from
//     another XCD's L2, i.e. most of a ~6.7 us step. The persistent engine
//     keeps parameters, momentum and the epoch's sampler indices in LDS
//     across steps, so a step costs only its compute and the all-reduce.
// Every configuration is a template instantiation (hidden layer / loss /
// update+all-reduce mode) with 32-bit index math: no runtime branching on the
// configuration in the executed path.
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include <time.h>
#include "sampler.h"

namespace ptdt {
namespace {

enum Mode : int { kNone = 0, kPre = 1, kArPost = 2, kArOnly = 3 };

__device__ __forceinline__ float sgd_one(float p, float g, float* mom, int i, bool first, float lr, float mu,
                                         float damp, float wd, int nesterov) {
  float d = g + wd * p;
  if (mom != nullptr && mu != 0.f) {
    const float buf = first ? d : mu * mom[i] + (1.f - damp) * d;
    mom[i] = buf;
    d = nesterov ? d + mu * buf : buf;
  }
  return p - lr * d;
}

// dot(x[0:n], w[0:n]) from LDS; 16-B reads when both rows are 16-B aligned.
__device__ __forceinline__ float dot_lds(const float* x, const float* w, int n, bool vec4) {
  float acc0 = 0.f, acc1 = 0.f;
  int k = 0;
  if (vec4) {
    for (; k + 4 <= n; k += 4) {
      const float4 xv = *reinterpret_cast<const float4*>(x + k);
      const float4 wv = *reinterpret_cast<const float4*>(w + k);
      acc0 = fmaf(xv.x, wv.x, acc0);
      acc1 = fmaf(xv.y, wv.y, acc1);
      acc0 = fmaf(xv.z, wv.z, acc0);
      acc1 = fmaf(xv.w, wv.w, acc1);
    }
  }
  for (; k < n; ++k) acc0 = fmaf(x[k], w[k], acc0);
  return acc0 + acc1;
}


struct Dims {
  int B, Din, H, Dout, Dh, nW1, nb1, nW2, nb2, np;
  __device__ __host__ Dims(int B_, int Din_, int H_, int Dout_, bool bias) : B(B_), Din(Din_), H(H_), Dout(Dout_) {
    Dh = H > 0 ? H : Din;
    nW1 = H > 0 ? H * Din : 0;
    nb1 = (H > 0 && bias) ? H : 0;
    nW2 = Dout * Dh;
    nb2 = bias ? Dout : 0;
    np = nW1 + nb1 + nW2 + nb2;
  }
};

// LDS scratch used by the step body
struct Scratch {
  float *xs, *as, *zs, *ds, *ys, *red;
};

// gather rows sel[0:B) of (X, Y) into LDS
template <int LOSS>
__device__ __forceinline__ void gather_batch(const FusedMlpArgs& a, const Dims& d, const int* sel, const Scratch& s,
                                             int tid, int NT) {
  const auto X = gptr(a.X);
  const int ldx = a.ldx > 0 ? a.ldx : d.Din;
  for (int e = tid; e < d.B * d.Din; e += NT) {
    const int b = e / d.Din, k = e - b * d.Din;
    s.xs[e] = X[(int64_t)sel[b] * ldx + k];
  }
  if constexpr (LOSS != kLossCEIndex) {
    const auto Yf = gptr(a.Yf);
    for (int e = tid; e < d.B * d.Dout; e += NT) {
      const int b = e / d.Dout, c = e - b * d.Dout;
      s.ys[e] = Yf[(int64_t)sel[b] * d.Dout + c];
    }
  } else {
    const auto Yi = gptr(a.Yi);
    int* yl = reinterpret_cast<int*>(s.ys);
    for (int b = tid; b < d.B; b += NT) yl[b] = (int)Yi[sel[b]];
  }
}

// out[e] = sum_{r<R} term(e, r) for e < E, each output reduced by a group of G
// adjacent lanes (G | 16): lane g of a group takes r = g, g+G, ... with four
// independent accumulators (so LDS loads overlap instead of forming one
// dependent chain), then log2(G) DPP adds inside the group. Replaces
// one-thread-per-output serial loops whose dependent LDS loads made the step
// latency-bound (profiles/).
// runtime group size (1, 2, 4, 8, 16): uniform branches, one code copy
__device__ __forceinline__ float group_sum_rt(float v, int G) {
  if (G >= 2) v += dpp_f<kDppXor1>(v);
  if (G >= 4) v += dpp_f<kDppXor2>(v);
  if (G >= 8) v += dpp_f<kDppHalfMirror>(v);
  if (G >= 16) v += dpp_f<kDppMirror>(v);
  return v;
}

template <typename Term, typename Store>
__device__ __forceinline__ void group_reduce(int G, int E, int R, Term term, Store store, int tid, int NT) {
  const int g = tid & (G - 1);
  const int per = NT / G;
  // every lane runs the same number of outer iterations so the DPP adds see a full wave
  const int rounds = (E + per - 1) / per;
  for (int it = 0; it < rounds; ++it) {
    const int e = it * per + tid / G;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    if (e < E) {
      int r = g;
      for (; r + 3 * G < R; r += 4 * G) {
        a0 += term(e, r);
        a1 += term(e, r + G);
        a2 += term(e, r + 2 * G);
        a3 += term(e, r + 3 * G);
      }
      for (; r < R; r += G) a0 += term(e, r);
    }
    const float v = group_sum_rt((a0 + a1) + (a2 + a3), G);
    if (e < E && g == 0) store(e, v);
  }
}

// out[e] = dot(x_row(e), w_row(e)) of length R with groups of G lanes, each
// lane owning contiguous 4-float chunks (ds_read_b128) when vec4 holds.
template <typename XRow, typename WRow, typename Store>
__device__ __forceinline__ void group_dot(int G, int E, int R, bool vec4, XRow xrow, WRow wrow, Store store, int tid,
                                          int NT) {
  const int g = tid & (G - 1);
  const int per = NT / G;
  const int rounds = (E + per - 1) / per;
  for (int it = 0; it < rounds; ++it) {
    const int e = it * per + tid / G;
    float a0 = 0.f, a1 = 0.f;
    if (e < E) {
      const float* x = xrow(e);
      const float* w = wrow(e);
      int k;
      if (vec4) {
        for (k = 4 * g; k + 4 <= R; k += 4 * G) {
          const float4 xv = *reinterpret_cast<const float4*>(x + k);
          const float4 wv = *reinterpret_cast<const float4*>(w + k);
          a0 = fmaf(xv.x, wv.x, a0);
          a1 = fmaf(xv.y, wv.y, a1);
          a0 = fmaf(xv.z, wv.z, a0);
          a1 = fmaf(xv.w, wv.w, a1);
        }
        for (k = (R & ~3) + g; k < R; k += G) a0 = fmaf(x[k], w[k], a0);
      } else {
        for (k = g; k < R; k += G) a0 = fmaf(x[k], w[k], a0);
      }
    }
    const float v = group_sum_rt(a0 + a1, G);
    if (e < E && g == 0) store(e, v);
  }
}

// Lanes per output: spread a reduction over a lane group only while the
// outputs alone cannot occupy the workgroup (E * G <= NT) and each lane keeps
// >= 2 terms; with enough outputs (the MLP's hidden layer) one lane per output
// with 16-B LDS reads is cheaper than any shuffle tree.
__device__ __forceinline__ int pick_group(int E, int R, int NT, int min_terms = 4) {
  int g = 1;
  while (g < 16 && E * (g * 2) <= NT && R >= min_terms * g * 2) g *= 2;
  return g;
}

// Diagnostic phase timers (thread 0, s_memtime cycles); `on` is false in
// production launches, so every tick is one uniform branch.
struct Stamps {
  bool on = false;
  int64_t prev = 0;
  int64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  __device__ __forceinline__ void start() {
    if (on) prev = (int64_t)__builtin_amdgcn_s_memtime();
  }
  __device__ __forceinline__ void tick(int k) {
    if (on) {
      const int64_t t = (int64_t)__builtin_amdgcn_s_memtime();
      acc[k] += t - prev;
      prev = t;
    }
  }
};

// forward + loss + backward of one batch staged in LDS. Gradients (times
// grad_scale / loss denominator) go to gdst (accumulated when acc); the mean
// loss to *loss_out. Ends with every gdst write issued (no trailing barrier).
template <bool HID, int LOSS>
__device__ __forceinline__ void step_body(const FusedMlpArgs& a, const Dims& d, const float* Ps, const Scratch& s,
                                          float* gdst, bool acc, float* loss_out, int tid, int NT, Stamps& st) {
  const int B = d.B, Din = d.Din, H = d.H, Dout = d.Dout, Dh = d.Dh;
  const float* W1 = Ps;
  const float* b1 = Ps + d.nW1;
  const float* W2 = Ps + d.nW1 + d.nb1;
  const float* b2 = W2 + d.nW2;
  float *as = s.as, *zs = s.zs, *ds = s.ds;
  const float* xs = s.xs;
  const float* ys = s.ys;
  const bool bias1 = d.nb1 != 0, bias2 = d.nb2 != 0;

  // ---- forward
  if constexpr (HID) {
    const bool v_in = (Din & 3) == 0;
    group_dot(pick_group(B * H, Din, NT, 8), B * H, Din, v_in,
                        [&](int e) { return xs + (e / H) * Din; }, [&](int e) { return W1 + (e % H) * Din; },
                        [&](int e, float v) { as[e] = fmaxf(v + (bias1 ? b1[e % H] : 0.f), 0.f); }, tid, NT);
    __syncthreads();
  }
  const float* act = HID ? as : xs;
  {
    const bool v_out = (Dh & 3) == 0 && ((d.nW1 + d.nb1) & 3) == 0;
    group_dot(pick_group(B * Dout, Dh, NT, 8), B * Dout, Dh, v_out,
                        [&](int e) { return act + (e / Dout) * Dh; }, [&](int e) { return W2 + (e % Dout) * Dh; },
                        [&](int e, float v) { zs[e] = v + (bias2 ? b2[e % Dout] : 0.f); }, tid, NT);
  }
  __syncthreads();
  st.tick(1);

  // ---- loss + dL/dlogits. Rows are spread over lanes; the loss SUM is only
  // needed for reporting, the gradient scale only needs the denominator
  // (B for soft CE, B*Dout for MSE, #valid rows for CE with ignore_index).
  float lsum = 0.f, cnt = 0.f;
  for (int b = tid; b < B; b += NT) {
    float* z = zs + b * Dout;
    if constexpr (LOSS == kLossMSE) {
      const float* t = ys + b * Dout;
      for (int c = 0; c < Dout; ++c) {
        const float df = z[c] - t[c];
        lsum = fmaf(df, df, lsum);
        z[c] = 2.f * df;
      }
    } else {
      float m = -INFINITY;
      for (int c = 0; c < Dout; ++c) m = fmaxf(m, z[c]);
      float se = 0.f;
      for (int c = 0; c < Dout; ++c) se += __expf(z[c] - m);
      const float lse = m + __logf(se);
      if constexpr (LOSS == kLossCESoft) {
        const float* t = ys + b * Dout;
        float tsum = 0.f, l = 0.f;
        for (int c = 0; c < Dout; ++c) {
          tsum += t[c];
          l -= t[c] * (z[c] - lse);
        }
        for (int c = 0; c < Dout; ++c) z[c] = __expf(z[c] - lse) * tsum - t[c];
        lsum += l;
      } else {
        const int y = reinterpret_cast<const int*>(ys)[b];
        if (y == a.ignore_index) {
          for (int c = 0; c < Dout; ++c) z[c] = 0.f;
        } else {
          lsum += lse - z[y];
          for (int c = 0; c < Dout; ++c) z[c] = __expf(z[c] - lse) - (c == y ? 1.f : 0.f);
          cnt += 1.f;
        }
      }
    }
  }
  float denom;
  if constexpr (LOSS == kLossCEIndex) {
    // the only case whose denominator depends on the data
    const float2 r2 = block_sum2(make_float2(lsum, cnt), s.red);
    lsum = r2.x;
    cnt = r2.y;
    denom = cnt > 0.f ? cnt : 1.f;
    if (tid == 0) *loss_out = cnt > 0.f ? lsum / denom : NAN;
  } else {
    denom = (LOSS == kLossMSE) ? (float)(B * Dout) : (float)B;
    // loss sum off the critical path: per-wave partials now, one lane adds them after the backward
    const float w = wave_sum(lsum);
    if ((tid & 63) == 0) s.red[16 + (tid >> 6)] = w;
    __syncthreads();
  }
  const float coef = a.grad_scale / denom;
  st.tick(2);

  // ---- backward, gradients into gdst
  float* gW1 = gdst;
  float* gb1 = gdst + d.nW1;
  float* gW2 = gdst + d.nW1 + d.nb1;
  float* gb2 = gW2 + d.nW2;
  group_reduce(pick_group(d.nW2 + d.nb2, B, NT), d.nW2 + d.nb2, B,
                    [&](int e, int b) {
                      if (e < d.nW2) {
                        const int c = e / Dh, j = e - c * Dh;
                        return zs[b * Dout + c] * act[b * Dh + j];
                      }
                      return zs[b * Dout + (e - d.nW2)];
                    },
                    [&](int e, float v) {
                      v *= coef;
                      if (e < d.nW2) gW2[e] = acc ? gW2[e] + v : v;
                      else gb2[e - d.nW2] = acc ? gb2[e - d.nW2] + v : v;
                    },
                    tid, NT);
  if constexpr (HID) {
    for (int e = tid; e < B * H; e += NT) {
      const int b = e / H, j = e - b * H;
      float sm = 0.f;
      if (as[e] > 0.f)
        for (int c = 0; c < Dout; ++c) sm = fmaf(zs[b * Dout + c], W2[c * H + j], sm);
      ds[e] = sm;
    }
    __syncthreads();
    group_reduce(pick_group(d.nW1 + d.nb1, B, NT), d.nW1 + d.nb1, B,
                      [&](int e, int b) {
                        if (e < d.nW1) {
                          const int j = e / Din, k = e - j * Din;
                          return ds[b * H + j] * xs[b * Din + k];
                        }
                        return ds[b * H + (e - d.nW1)];
                      },
                      [&](int e, float v) {
                        v *= coef;
                        if (e < d.nW1) gW1[e] = acc ? gW1[e] + v : v;
                        else gb1[e - d.nW1] = acc ? gb1[e - d.nW1] + v : v;
                      },
                      tid, NT);
  }
  if constexpr (LOSS != kLossCEIndex) {
    if (tid == 0) {
      float l = 0.f;
      for (int w = 0; w < (NT >> 6); ++w) l += s.red[16 + w];
      *loss_out = l / denom;
    }
  }
}

// Average `np` gradients held in LDS across ranks (in place). world == 1 is
// the identity: DDP over one rank averages nothing.
// PB: poll loads in flight per thread (16 for the 256-thread MFMA engine measured no
// faster than 8 at W = 2 and 4, and costs step-body VGPRs)
template <int PB = 8>
__device__ __forceinline__ void allreduce_lds(const XgmiArgs& ar, uint32_t seq, float* gs, float* tmp, int np,
                                              int tid, int NT, int* lds_flag = nullptr) {
  if (ar.world <= 1) return;
  xgmi_push(ar, seq, gs, np, tid, NT);
  xgmi_gather_lds<PB>(ar, seq, 0, np, tmp, tid, NT, lds_flag);
  __syncthreads();
  const float inv_w = 1.f / (float)ar.world;
  for (int i = tid; i < np; i += NT) gs[i] = xgmi_sum_lds(tmp, ar.world, np, i) * inv_w;
  __syncthreads();
}

// ------------------------------------------------------------------ per-step kernel
// Critical path = two dependent global round trips: (sampler indices || params,
// grads, opt state) -> barrier -> (dataset rows X, Y gathered by index) ->
// barrier; everything after runs out of LDS.
template <bool HID, int LOSS, int MODE>
__global__ void __launch_bounds__(1024) fused_mlp_step_kernel(FusedMlpArgs a) {
  extern __shared__ float lds[];
  constexpr bool AR = (MODE == kArPost || MODE == kArOnly);
  constexpr bool FY = LOSS != kLossCEIndex;
  const int tid = threadIdx.x, NT = blockDim.x;
  const Dims d(a.B, a.Din, HID ? a.H : 0, a.Dout, a.has_bias != 0);
  const int np = d.np, B = d.B;

  float* Ps = lds;
  Scratch s;
  s.xs = Ps + al4(np);
  s.as = s.xs + al4(B * d.Din);
  s.zs = s.as + al4(B * d.H);
  s.ds = s.zs + al4(B * d.Dout);
  s.ys = s.ds + al4(B * d.H);
  int* sidx = reinterpret_cast<int*>(s.ys + al4(FY ? B * d.Dout : B));
  s.red = reinterpret_cast<float*>(sidx + al4(B));
  float* gs = s.red + 32;              // [np] local grads (in-kernel all-reduce only)
  float* tmp = gs + al4(np);           // [world * np] staged peer contributions

  const bool first = (a.opt_step != nullptr) ? (*a.opt_step == 0) : false;
  uint32_t ar_seq = 0;
  XgmiArgs ar = a.ar;
  if constexpr (AR) {
    ar_seq = *a.ar.seq + 1u;
    if (ar.world > 1 && *a.ar.err != 0) ar.world = 1;  // a peer already timed out: do not wait again
  }

  // trip 1: sampler indices, params (with the deferred update of the previous step)
  for (int b = tid; b < B; b += NT) sidx[b] = a.idx ? a.idx[b] : b;
  if constexpr (MODE == kPre) {
    for (int i = tid; i < np; i += NT) {
      const float p = sgd_one(a.P[i], a.G[i], a.mom, i, first, a.lr, a.momentum, a.dampening, a.weight_decay,
                              a.nesterov);
      a.P[i] = p;
      Ps[i] = p;
    }
  } else {
    for (int i = tid; i < np; i += NT) Ps[i] = a.P[i];
  }
  __syncthreads();
  if constexpr (MODE == kPre) {
    if (tid == 0 && a.opt_step != nullptr) *a.opt_step += 1;
  }
  // trip 2: the batch rows
  gather_batch<LOSS>(a, d, sidx, s, tid, NT);
  __syncthreads();

  Stamps st;
  step_body<HID, LOSS>(a, d, Ps, s, AR ? gs : a.G, !AR && a.accumulate != 0, a.loss_out, tid, NT, st);

  if constexpr (AR) {
    __syncthreads();
    allreduce_lds(ar, ar_seq, gs, tmp, np, tid, NT);
    for (int i = tid; i < np; i += NT) {
      const float g = gs[i];
      a.G[i] = g;  // .grad holds the global average, as after DDP's finalize
      if constexpr (MODE == kArPost)
        a.P[i] = sgd_one(Ps[i], g, a.mom, i, first, a.lr, a.momentum, a.dampening, a.weight_decay, a.nesterov);
    }
    if (tid == 0) {
      if (ar.world > 1) *a.ar.seq = ar_seq;
      if (MODE == kArPost && a.opt_step != nullptr) *a.opt_step += 1;
    }
  }
}

// ------------------------------------------------------------------ persistent engine
// ---------------------------------------------------------------------------
// MFMA step body for Linear(Din, H)-ReLU-Linear(H, Dout) (the "toy MLP"):
// four waves, every product on v_mfma_f32_16x16x4f32 (exact fp32 multiply-adds)
// with LDS-staged operand tiles, instead of the LDS dot products of step_body.
// Shapes: B <= 32 rows, Din <= 32, H in {16, 32, 48, 64} (wave w owns hidden
// tile w), Dout <= 16. LDS matrices use padded row strides (H+8, 17) so the
// lanes reading a fragment hit at most 2 lanes per bank.
// Layout of v_mfma_f32_16x16x4f32: lane l supplies A[l%16][l/16] and
// B[l/16][l%16]; the result lane holds C[4*(l/16) + r][l%16], r = 0..3.
//   fwd1  A1 = relu(X W1^T + b1)       wave w: rows 0-31 x hidden 16w..16w+15
//   fwd2  Z2 = A1 W2^T + b2, loss,      waves 0/1: rows 16w..16w+15; the
//         dL/dZ2 in registers           softmax row reductions are DPP adds
//                                       inside one 16-lane DPP row
//   bwd   dW2 = dZ2^T A1, dA1 = dZ2 W2, dZ1 = dA1 * [A1 > 0], db1 (permlane
//         swaps across the 4 DPP rows), dW1 = dZ1^T X; db2 from fwd2's partials
typedef __attribute__((ext_vector_type(4))) float mf4;

__device__ __forceinline__ mf4 mfma4(float a, float b, mf4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_f<kDppXor1>(v));
  v = fmaxf(v, dpp_f<kDppXor2>(v));
  v = fmaxf(v, dpp_f<kDppHalfMirror>(v));
  return fmaxf(v, dpp_f<kDppMirror>(v));
}
// sum of the 4 lanes l%16 == c (one per DPP row), in all of them
__device__ __forceinline__ float across_rows_sum(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
  v = __int_as_float(p[0]) + __int_as_float(p[1]);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(q[0]) + __int_as_float(q[1]);
}

constexpr int kMfThreads = 256;
constexpr int kMfRows = 32;
constexpr int kMfZ = 17;  // dz row stride (Dout <= 16)
// a1 / dz1 / w2p row stride: fragments are read both with lanes along rows (c*la + g)
// and along columns (g*la + c); H + 8 keeps both at <= 2-way bank conflicts
__host__ __device__ constexpr int kMfPad(int H) { return H + 8; }

__host__ __device__ inline bool mlp_mfma_shape_ok(int B, int Din, int H, int Dout) {
  return B >= 1 && B <= kMfRows && Din >= 1 && Din <= 32 && H >= 16 && H <= 64 && H % 16 == 0 && Dout >= 1 &&
         Dout <= 16;
}

// Operands of a whole K chain are loaded into registers first (all LDS reads in
// flight together), then the MFMAs run as two independent accumulator chains:
// the step is otherwise a series of LDS-latency + MFMA-latency round trips.
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS traffic,
// not for its global loads, so the next step's register prefetch stays in flight
// (__syncthreads' workgroup fence would drain it -- cdna_hip_programming.md §5).
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

template <int NK>
__device__ __forceinline__ mf4 mfma_chain(const float (&av)[NK], const float (&bv)[NK]) {
  mf4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < NK; k += 2) {
    c0 = mfma4(av[k], bv[k], c0);
    if (k + 1 < NK) c1 = mfma4(av[k + 1], bv[k + 1], c1);
  }
  return c0 + c1;
}

template <int LOSS, int HT>
__device__ __forceinline__ void step_body_mfma(const FusedMlpArgs& a, const Dims& d, const float* Ps,
                                               const Scratch& s, float* gdst, float* loss_out, int tid, Stamps& st) {
  constexpr int H = 16 * HT, la = kMfPad(H);
  const int B = d.B, Din = d.Din, Dout = d.Dout;
  const float* W1 = Ps;
  const float* b1 = Ps + d.nW1;
  const float* W2 = Ps + d.nW1 + d.nb1;
  const float* b2 = W2 + d.nW2;
  const bool bias1 = d.nb1 != 0, bias2 = d.nb2 != 0;
  float* a1 = s.as;   // [32][la] relu(Z1), rows >= B zero
  float* dz = s.zs;   // [32][17]  dL/dZ2, scaled; rows >= B and cols >= Dout zero
  float* dz1 = s.ds;  // [32][la] dL/dZ1
  float* w2p = s.ds;  // [Dout][la] W2 copy for fwd2 (dead before dz1 is written)
  float* red = s.red; // [64]: loss partials, db2 partials
  const float* xs = s.xs;
  const int w = tid >> 6, l = tid & 63, g = l >> 4, c = l & 15;
  float* gW1 = gdst;
  float* gb1 = gdst + d.nW1;
  float* gW2 = gdst + d.nW1 + d.nb1;
  float* gb2 = gW2 + d.nW2;

  {  // W2 copy: all reads in flight, then the writes (Dout * H <= 4 * kMfThreads)
    float t[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + q * kMfThreads;
      t[q] = e < Dout * H ? W2[e] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + q * kMfThreads;
      if (e < Dout * H) w2p[(e / H) * la + (e % H)] = t[q];
    }
  }
  // ---- fwd1: wave w -> hidden tile w, both 16-row tiles (K = Din: 5 steps up to 20, else 8, masked)
  if (w < HT) {
    const int h = 16 * w + c;
    const float bb = bias1 ? b1[h] : 0.f;
    mf4 z0, z1;
    auto fwd1 = [&](auto nk) {
      constexpr int NK = decltype(nk)::value;
      float bv[NK], av0[NK], av1[NK];
#pragma unroll
      for (int q = 0; q < NK; ++q) {
        const int k = 4 * q + g;
        const bool kin = k < Din;
        bv[q] = kin ? W1[h * Din + k] : 0.f;
        av0[q] = (kin && c < B) ? xs[c * Din + k] : 0.f;
        av1[q] = (kin && 16 + c < B) ? xs[(16 + c) * Din + k] : 0.f;
      }
      z0 = mfma_chain<NK>(av0, bv);
      z1 = mfma_chain<NK>(av1, bv);
    };
    if (Din <= 20) fwd1(std::integral_constant<int, 5>{});
    else fwd1(std::integral_constant<int, 8>{});
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int r0 = 4 * g + r, r1 = 16 + 4 * g + r;
      a1[r0 * la + h] = r0 < B ? fmaxf(z0[r] + bb, 0.f) : 0.f;
      a1[r1 * la + h] = r1 < B ? fmaxf(z1[r] + bb, 0.f) : 0.f;
    }
  }
  lds_sync();
  // ---- fwd2 + loss + dL/dZ2 (waves 0, 1: row tile w)
  if (w < 2) {
    float av[4 * HT], bv[4 * HT];
#pragma unroll
    for (int q = 0; q < 4 * HT; ++q) {
      av[q] = a1[(16 * w + c) * la + 4 * q + g];
      bv[q] = c < Dout ? w2p[c * la + 4 * q + g] : 0.f;
    }
    const mf4 acc = mfma_chain<4 * HT>(av, bv);
    st.tick(1);
    const bool col = c < Dout;
    const float bz = (bias2 && col) ? b2[c] : 0.f;
    float denom;
    if constexpr (LOSS == kLossCEIndex) {
      const int* yl = reinterpret_cast<const int*>(s.ys);
      const bool v = l < B && yl[l] != a.ignore_index;
      denom = (float)__builtin_popcountll(__ballot(v));
    } else {
      denom = (LOSS == kLossMSE) ? (float)(B * Dout) : (float)B;
    }
    const float coef = a.grad_scale / (denom > 0.f ? denom : 1.f);
    float lsum = 0.f, csum = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * w + 4 * g + r;
      const bool rv = row < B;
      const float z = acc[r] + bz;
      float dzv = 0.f;
      if constexpr (LOSS == kLossMSE) {
        const float t = (rv && col) ? s.ys[row * Dout + c] : 0.f;
        const float df = (rv && col) ? z - t : 0.f;
        lsum = fmaf(df, df, lsum);
        dzv = 2.f * df;
      } else {
        const float m = row16_max(col ? z : -INFINITY);
        const float ez = col ? __expf(z - m) : 0.f;
        const float lse = m + __logf(group_sum<16>(ez));
        if constexpr (LOSS == kLossCESoft) {
          const float t = (rv && col) ? s.ys[row * Dout + c] : 0.f;
          const float tsum = group_sum<16>(t);
          const float lrow = group_sum<16>(col ? -t * (z - lse) : 0.f);
          if (c == 0) lsum += lrow;
          dzv = (rv && col) ? __expf(z - lse) * tsum - t : 0.f;
        } else {
          const int y = rv ? reinterpret_cast<const int*>(s.ys)[row] : -1;
          const bool ok = rv && y != a.ignore_index;
          if (ok && c == y) lsum += lse - z;
          dzv = (ok && col) ? __expf(z - lse) - (c == y ? 1.f : 0.f) : 0.f;
        }
      }
      dzv *= coef;
      dz[row * kMfZ + c] = dzv;
      csum += dzv;
    }
    const float lw = wave_sum(lsum);
    const float cs = across_rows_sum(csum);  // this row tile's column sums (db2 partials)
    if (l == 0) red[w] = lw;
    if (l < 16) red[16 + 16 * w + l] = cs;
    if (tid == 0) red[2] = denom;
  }
  lds_sync();
  st.tick(2);
  if (tid == 0) {
    if constexpr (LOSS == kLossCEIndex) *loss_out = red[2] > 0.f ? (red[0] + red[1]) / red[2] : NAN;
    else *loss_out = (red[0] + red[1]) / red[2];
  }
  // ---- backward: dW2, dA1 -> dZ1, db1, db2 (wave w: hidden tile w)
  if (w < HT) {
    const int h = 16 * w + c;
    float av[8], bv[8], ad0[4], ad1[4], bw[4], m0[4], m1[4];
#pragma unroll
    for (int q = 0; q < 8; ++q) {  // dW2[o][h] = sum_row dz[row][o] a1[row][h]
      av[q] = dz[(4 * q + g) * kMfZ + c];
      bv[q] = a1[(4 * q + g) * la + h];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // dA1[row][h] = sum_o dz[row][o] W2[o][h]
      const int o = 4 * q + g;
      ad0[q] = dz[c * kMfZ + o];
      ad1[q] = dz[(16 + c) * kMfZ + o];
      bw[q] = o < Dout ? W2[o * H + h] : 0.f;
      m0[q] = a1[(4 * g + q) * la + h];
      m1[q] = a1[(16 + 4 * g + q) * la + h];
    }
    const mf4 gw2 = mfma_chain<8>(av, bv);
    const mf4 da0 = mfma_chain<4>(ad0, bw), da1 = mfma_chain<4>(ad1, bw);
    float db = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = 4 * g + r;
      if (o < Dout) gW2[o * H + h] = gw2[r];
      const float v0 = m0[r] > 0.f ? da0[r] : 0.f, v1 = m1[r] > 0.f ? da1[r] : 0.f;
      dz1[(4 * g + r) * la + h] = v0;
      dz1[(16 + 4 * g + r) * la + h] = v1;
      db += v0 + v1;
    }
    db = across_rows_sum(db);
    if (bias1 && l < 16) gb1[h] = db;
  }
  if (bias2 && tid < Dout) gb2[tid] = red[16 + tid] + red[32 + tid];
  lds_sync();
  // ---- dW1[h][k] = sum_row dz1[row][h] x[row][k]
  if (w < HT) {
    float av[8], bv0[8], bv1[8];
    const bool two = Din > 16;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int row = 4 * q + g;
      av[q] = dz1[row * la + 16 * w + c];
      bv0[q] = (row < B && c < Din) ? xs[row * Din + c] : 0.f;
      bv1[q] = (two && row < B && 16 + c < Din) ? xs[row * Din + 16 + c] : 0.f;
    }
    const mf4 g0 = mfma_chain<8>(av, bv0);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (c < Din) gW1[(16 * w + 4 * g + r) * Din + c] = g0[r];
    if (two) {
      const mf4 g1 = mfma_chain<8>(av, bv1);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (16 + c < Din) gW1[(16 * w + 4 * g + r) * Din + 16 + c] = g1[r];
    }
  }
}

// Per-thread register prefetch of the NEXT step's batch rows: the global loads
// are issued before this step's compute and written to the other LDS batch
// buffer after it, so the gather latency is off the critical path.
constexpr int kPf = 4;  // prefetched elements per thread (B*Din and B*Dout must be <= kPf * blockDim)

template <int LOSS>
struct Prefetch {
  float x[kPf];
  float y[kPf];
  int yi[kPf];
  int xb[kPf], xk[kPf];  // (row, column) of element tid + q * NT: fixed per thread, divided once
  int yb[kPf], yk[kPf];
  __device__ __forceinline__ void setup(int Din, int Dout, int tid, int NT) {
#pragma unroll
    for (int q = 0; q < kPf; ++q) {
      const int e = tid + q * NT;
      xb[q] = e / Din;
      xk[q] = e - xb[q] * Din;
      yb[q] = e / Dout;
      yk[q] = e - yb[q] * Dout;
    }
  }
  __device__ __forceinline__ void issue(const FusedMlpArgs& a, const int* sel, int B, int Din, int Dout, int tid,
                                        int NT) {
    const auto X = gptr(a.X);
    const int ldx = a.ldx > 0 ? a.ldx : Din;
#pragma unroll
    for (int q = 0; q < kPf; ++q) {
      const int e = tid + q * NT;
      if (xb[q] < B) x[q] = X[(int64_t)sel[xb[q]] * ldx + xk[q]];
      if constexpr (LOSS != kLossCEIndex) {
        if (yb[q] < B) y[q] = gptr(a.Yf)[(int64_t)sel[yb[q]] * Dout + yk[q]];
      } else {
        if (e < B) yi[q] = (int)gptr(a.Yi)[sel[e]];
      }
    }
  }
  __device__ __forceinline__ void land(float* xs, float* ys, int B, int Din, int Dout, int tid, int NT) const {
#pragma unroll
    for (int q = 0; q < kPf; ++q) {
      const int e = tid + q * NT;
      if (e < B * Din) xs[e] = x[q];
      if constexpr (LOSS != kLossCEIndex) {
        if (e < B * Dout) ys[e] = y[q];
      } else {
        if (e < B) reinterpret_cast<int*>(ys)[e] = yi[q];
      }
    }
  }
};

// MF: 0 = LDS dot-product step body (1024 threads); 1..4 = the MFMA body for H = 16 * MF
// (one hidden width per instantiation keeps the per-step code small in the instruction cache)
template <bool HID, int LOSS, int MF>
__global__ void __launch_bounds__(MF ? kMfThreads : 1024) fused_mlp_persistent_kernel(FusedMlpArgs a, PersistArgs pa) {
  extern __shared__ float lds[];
  constexpr bool FY = LOSS != kLossCEIndex;
  const int tid = threadIdx.x, NT = blockDim.x;
  const Dims full(a.B, a.Din, HID ? a.H : 0, a.Dout, a.has_bias != 0);
  const int np = full.np, B = full.B;
  const bool use_mom = a.mom != nullptr && a.momentum != 0.f;
  const int ylen = al4(FY ? B * full.Dout : B);

  float* Ps = lds;                                 // live parameters
  float* Ms = Ps + al4(np);                        // live momentum
  float* gs = Ms + al4(np);                        // grads of the current step
  // double-buffered batch: buffer k at xs0 + k * xstride (offset arithmetic keeps the
  // pointers provably LDS -> ds_* instructions, never flat_*)
  float* const xs0 = gs + al4(np);
  const int xstride = al4(B * full.Din);
  float* const ys0 = xs0 + 2 * xstride;
  const int ystride = ylen;
  Scratch s;
  s.as = ys0 + 2 * ystride;
  if constexpr (MF != 0) {  // MFMA body: padded row strides, 32 rows
    s.zs = s.as + al4(kMfRows * kMfPad(full.H));
    s.ds = s.zs + al4(kMfRows * kMfZ);
    s.red = s.ds + al4(kMfRows * kMfPad(full.H));
  } else {
    s.zs = s.as + al4(B * full.H);
    s.ds = s.zs + al4(B * full.Dout);
    s.red = s.ds + al4(B * full.H);
  }
  float* tmp = s.red + (MF ? 64 : 32);             // [world * np]
  int* const eb0 = reinterpret_cast<int*>(tmp + al4((a.ar.world > 1 ? a.ar.world : 1) * np));  // epoch lists
  const int estride = al4(pa.num_samples);
  auto ebuf = [&](int e) { return eb0 + (e & 1) * estride; };
  int* lds_err = eb0 + 2 * estride;               // set by a timed-out poll
  if (tid == 0) *lds_err = 0;

  // ---- load resident state; index lists of the current and the next epoch
  for (int i = tid; i < np; i += NT) {
    Ps[i] = a.P[i];
    Ms[i] = use_mom ? a.mom[i] : 0.f;
  }
  int epoch = pa.cursor[0], j = pa.cursor[1];
  const int steps_per_epoch = (pa.num_samples + B - 1) / B;
  int opt_step = a.opt_step ? *a.opt_step : 0;
  uint32_t seq = a.ar.world > 1 ? *a.ar.seq : 0u;
  const ListCache lc{pa.lcache, pa.ltag, estride};
  rank_epoch_indices_or(given_list(pa, epoch), ebuf(epoch), (uint32_t)pa.N, pa.W, pa.rank, pa.num_samples, pa.seed, epoch, pa.shuffle,
                     tid, NT, lc);
  rank_epoch_indices_or(given_list(pa, epoch + 1), ebuf(epoch + 1), (uint32_t)pa.N, pa.W, pa.rank, pa.num_samples, pa.seed, epoch + 1,
                     pa.shuffle, tid, NT, lc);
  __syncthreads();
  if (tid == 0 && pa.idx == nullptr) {
    list_cache_publish(lc, epoch);
    list_cache_publish(lc, epoch + 1);
  }
  const bool pf_ok = B * full.Din <= kPf * NT && B * (FY ? full.Dout : 1) <= kPf * NT;
  auto batch_size = [&](int jj) { return pa.num_samples - jj * B < B ? pa.num_samples - jj * B : B; };
  {  // first batch (synchronous)
    Scratch s0 = s;
    s0.xs = xs0;
    s0.ys = ys0;
    const Dims d0(batch_size(j), full.Din, full.H, full.Dout, a.has_bias != 0);
    gather_batch<LOSS>(a, d0, ebuf(epoch) + j * B, s0, tid, NT);
  }
  __syncthreads();

  Prefetch<LOSS> pf;
  pf.setup(full.Din, full.Dout, tid, NT);
  Stamps st;
  st.on = pa.stamps != nullptr && tid == 0;
  const int64_t t_begin = st.on ? (int64_t)__builtin_amdgcn_s_memtime() : 0;
  const int64_t r_begin = st.on ? (int64_t)__builtin_amdgcn_s_memrealtime() : 0;
  st.start();

  for (int step = 0; step < pa.n_steps; ++step) {
    const int cur = step & 1;
    // next step's position, and the epoch after next computed one epoch ahead
    int nj = j + 1, ne = epoch;
    if (nj == steps_per_epoch) {
      nj = 0;
      ++ne;
    }
    if (j == 0 && step > 0) {
      rank_epoch_indices_or(given_list(pa, epoch + 1), ebuf(epoch + 1), (uint32_t)pa.N, pa.W, pa.rank, pa.num_samples, pa.seed, epoch + 1,
                         pa.shuffle, tid, NT, lc);
      __syncthreads();
      if (tid == 0 && pa.idx == nullptr) list_cache_publish(lc, epoch + 1);
    }
    st.tick(6);
    const int nb = batch_size(nj);
    const bool have_next = step + 1 < pa.n_steps;
    if (pf_ok && have_next) pf.issue(a, ebuf(ne) + nj * B, nb, full.Din, full.Dout, tid, NT);
    st.tick(0);

    s.xs = xs0 + cur * xstride;
    s.ys = ys0 + cur * ystride;
    const Dims d(batch_size(j), full.Din, full.H, full.Dout, a.has_bias != 0);
    if constexpr (MF != 0) {
      step_body_mfma<LOSS, MF>(a, d, Ps, s, gs, pa.losses + step, tid, st);
      lds_sync();  // grads visible; the prefetch is still in flight
    } else {
      step_body<HID, LOSS>(a, d, Ps, s, gs, false, pa.losses + step, tid, NT, st);
      __syncthreads();
    }
    st.tick(3);
    seq += 1u;
    allreduce_lds(a.ar, seq, gs, tmp, np, tid, NT, lds_err);
    st.tick(4);
    const bool first = opt_step == 0;
    {  // 4 independent updates per iteration: their LDS loads overlap instead of chaining
      int i = tid;
      for (; i + 3 * NT < np; i += 4 * NT) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          Ps[i + u * NT] = sgd_one(Ps[i + u * NT], gs[i + u * NT], use_mom ? Ms : nullptr, i + u * NT, first, a.lr,
                                   a.momentum, a.dampening, a.weight_decay, a.nesterov);
      }
      for (; i < np; i += NT)
        Ps[i] = sgd_one(Ps[i], gs[i], use_mom ? Ms : nullptr, i, first, a.lr, a.momentum, a.dampening,
                        a.weight_decay, a.nesterov);
    }
    ++opt_step;
    // land the prefetched batch in the other buffer (last read two steps ago)
    if (have_next) {
      if (pf_ok) {
        pf.land(xs0 + (cur ^ 1) * xstride, ys0 + (cur ^ 1) * ystride, nb, full.Din, full.Dout, tid, NT);
      } else {
        Scratch sn = s;
        sn.xs = xs0 + (cur ^ 1) * xstride;
        sn.ys = ys0 + (cur ^ 1) * ystride;
        const Dims dn(nb, full.Din, full.H, full.Dout, a.has_bias != 0);
        gather_batch<LOSS>(a, dn, ebuf(ne) + nj * B, sn, tid, NT);
      }
    }
    j = nj;
    epoch = ne;
    __syncthreads();
    st.tick(5);
    if (*lds_err) break;  // a peer vanished: stop instead of timing out on every remaining step
  }

  // ---- write back resident state
  for (int i = tid; i < np; i += NT) {
    a.P[i] = Ps[i];
    a.G[i] = gs[i];
    if (use_mom) a.mom[i] = Ms[i];
  }
  if (tid == 0) {
    pa.cursor[0] = epoch;
    pa.cursor[1] = j;
    if (a.opt_step) *a.opt_step = opt_step;
    if (a.ar.world > 1) *a.ar.seq = seq;
    if (st.on) {
      // [0] prefetch issue, [1] forward, [2] loss, [3] backward, [4] all-reduce, [5] sgd+land, [6] epoch indices
      for (int k = 0; k < 7; ++k) pa.stamps[k] += st.acc[k];
      pa.stamps[7] += (int64_t)__builtin_amdgcn_s_memtime() - t_begin;
      pa.stamps[8] += (int64_t)__builtin_amdgcn_s_memrealtime() - r_begin;
    }
  }
}

template <bool HID, int LOSS>
const void* pick_mode(int mode) {
  switch (mode) {
    case kPre: return (const void*)fused_mlp_step_kernel<HID, LOSS, kPre>;
    case kArPost: return (const void*)fused_mlp_step_kernel<HID, LOSS, kArPost>;
    case kArOnly: return (const void*)fused_mlp_step_kernel<HID, LOSS, kArOnly>;
    default: return (const void*)fused_mlp_step_kernel<HID, LOSS, kNone>;
  }
}

template <bool HID>
const void* pick_loss(int loss, int mode) {
  switch (loss) {
    case kLossCEIndex: return pick_mode<HID, kLossCEIndex>(mode);
    case kLossMSE: return pick_mode<HID, kLossMSE>(mode);
    default: return pick_mode<HID, kLossCESoft>(mode);
  }
}

template <bool HID, int MF = 0>
const void* pick_persist(int loss) {
  switch (loss) {
    case kLossCEIndex: return (const void*)fused_mlp_persistent_kernel<HID, kLossCEIndex, MF>;
    case kLossMSE: return (const void*)fused_mlp_persistent_kernel<HID, kLossMSE, MF>;
    default: return (const void*)fused_mlp_persistent_kernel<HID, kLossCESoft, MF>;
  }
}

const void* pick_persist_mfma(int loss, int H) {
  switch (H >> 4) {
    case 1: return pick_persist<true, 1>(loss);
    case 2: return pick_persist<true, 2>(loss);
    case 3: return pick_persist<true, 3>(loss);
    default: return pick_persist<true, 4>(loss);
  }
}

bool mfma_engine(const FusedMlpArgs& a, const PersistArgs& p) {
  return a.H > 0 && (p.variant == kPersistAuto || p.variant == kPersistMfma) &&
         mlp_mfma_shape_ok(a.B, a.Din, a.H, a.Dout) && !(p.variant == kPersistAuto && mlp_tp_supported(a, p));
}

hipError_t check_dims(const FusedMlpArgs& a) {
  if (a.B <= 0 || a.Din <= 0 || a.Dout <= 0 || a.H < 0) return hipErrorInvalidValue;
  const int64_t widest = a.Din > a.H ? (a.Din > a.Dout ? a.Din : a.Dout) : (a.H > a.Dout ? a.H : a.Dout);
  if ((int64_t)a.B * widest >= (1ll << 30)) return hipErrorInvalidValue;
  return hipSuccess;
}

int64_t num_params(const FusedMlpArgs& a) {
  const int Dh = a.H > 0 ? a.H : a.Din;
  return (a.H > 0 ? (int64_t)a.H * a.Din + (a.has_bias ? a.H : 0) : 0) + (int64_t)a.Dout * Dh +
         (a.has_bias ? a.Dout : 0);
}

}  // namespace

size_t fused_mlp_lds_bytes(int B, int Din, int H, int Dout) {
  const int Dh = H > 0 ? H : Din;
  const int np = (H > 0 ? H * Din + H : 0) + Dout * Dh + Dout;
  const int64_t fl = (int64_t)al4(np) + al4(B * Din) + 2 * al4(B * H) + 2 * al4(B * Dout) + al4(B) + al4(B) + 32 +
                     al4(np) + (int64_t)kXgmiMaxRanks * np;
  return (size_t)fl * sizeof(float);
}

size_t fused_mlp_persistent_lds_bytes(int B, int Din, int H, int Dout, int num_samples, int world) {
  const int Dh = H > 0 ? H : Din;
  const int np = (H > 0 ? H * Din + H : 0) + Dout * Dh + Dout;
  const int64_t common = 3 * (int64_t)al4(np) + 2 * al4(B * Din) + 2 * al4(B * Dout > B ? B * Dout : B) +
                         al4((world > 1 ? world : 1) * np) + 2 * al4(num_samples) + 4;
  int64_t fl = common + 2 * al4(B * H) + al4(B * Dout) + 32;
  if (H > 0 && mlp_mfma_shape_ok(B, Din, H, Dout)) {  // the MFMA body's padded scratch (the larger of the two)
    const int64_t mf = common + 2 * al4(kMfRows * kMfPad(H)) + al4(kMfRows * kMfZ) + 64;
    if (mf > fl) fl = mf;
  }
  return (size_t)fl * sizeof(float);
}

hipError_t fused_mlp_step(const FusedMlpArgs& a, hipStream_t s) {
  PTDT_HIP_CHECK(check_dims(a));
  const size_t lds = fused_mlp_lds_bytes(a.B, a.Din, a.H, a.Dout);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  int mode = a.update_mode == 1 ? kPre : kNone;
  if (a.ar.world > 0) {
    if (num_params(a) > a.ar.max_elems || a.update_mode == 1 || a.accumulate) return hipErrorInvalidValue;
    mode = a.update_mode == 2 ? kArPost : kArOnly;
  }
  const void* fn = a.H > 0 ? pick_loss<true>(a.loss_kind, mode) : pick_loss<false>(a.loss_kind, mode);
  if (lds > 64 * 1024)
    PTDT_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int threads = a.H > 0 ? 1024 : 256;
  void* args[] = {const_cast<FusedMlpArgs*>(&a)};
  return hipLaunchKernel(fn, dim3(1), dim3(threads), args, lds, s);
}

hipError_t fused_mlp_persistent_prepare(const FusedMlpArgs& a, const PersistArgs& p, PersistLaunch* out) {
  PTDT_HIP_CHECK(check_dims(a));
  if (a.update_mode != 2 || a.accumulate || p.cursor == nullptr || p.losses == nullptr || p.num_samples <= 0 ||
      p.N <= 0 || p.W <= 0 || p.rank < 0 || p.rank >= p.W)
    return hipErrorInvalidValue;
  if (a.ar.world > 1 && (num_params(a) > a.ar.max_elems || a.ar.world != p.W || a.ar.rank != p.rank))
    return hipErrorInvalidValue;
  if (p.variant != kPersistWorkgroup && p.variant != kPersistMfma && p.variant != kPersistTp &&
      p.variant != kPersistTpBf16 && linear_wave_supported(a, p))
    return linear_wave_prepare(a, p, out);
  if ((p.variant == kPersistAuto || p.variant == kPersistTp || p.variant == kPersistTpBf16) && a.H > 0 &&
      mlp_tp_supported(a, p))
    return mlp_tp_prepare(a, p, out);
  if (p.variant >= kPersistWave && p.variant != kPersistMfma) return hipErrorInvalidValue;
  const size_t lds = fused_mlp_persistent_lds_bytes(a.B, a.Din, a.H, a.Dout, p.num_samples, a.ar.world);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const bool mf = mfma_engine(a, p);
  if (p.variant == kPersistMfma && !mf) return hipErrorInvalidValue;
  const void* fn = mf ? pick_persist_mfma(a.loss_kind, a.H)
                      : (a.H > 0 ? pick_persist<true>(a.loss_kind) : pick_persist<false>(a.loss_kind));
  if (lds > 64 * 1024)
    PTDT_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  out->fn = fn;
  out->threads = mf ? kMfThreads : (a.H > 0 ? 1024 : 256);
  out->lds = lds;
  out->a = a;
  out->p = p;
  return hipSuccess;
}

hipError_t persistent_launch(PersistLaunch& L, int n_steps, int64_t cursor_host_pos, hipStream_t s, int start_e,
                             int start_j) {
  if (n_steps <= 0) return hipSuccess;
  if (L.fn == nullptr) return hipErrorInvalidValue;
  if (L.p.idx != nullptr) {  // explicit lists cover epochs [idx_e0, idx_e0 + idx_epochs) only
    const int64_t S = (L.p.num_samples + L.a.B - 1) / L.a.B;
    if (cursor_host_pos < (int64_t)L.p.idx_e0 * S || cursor_host_pos + n_steps > (int64_t)(L.p.idx_e0 + L.p.idx_epochs) * S)
      return hipErrorInvalidValue;
  }
  L.p.n_steps = n_steps;
  L.p.cursor_host_pos = cursor_host_pos;
  L.p.has_start = start_e >= 0 ? 1 : 0;
  L.p.start_e = start_e;
  L.p.start_j = start_j;
  void* args[] = {&L.a, &L.p};
  timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  const hipError_t e = hipLaunchKernel(L.fn, dim3(1), dim3(L.threads), args, L.lds, s);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  L.host_ns[0] = (int64_t)t0.tv_sec * 1000000000 + t0.tv_nsec;
  L.host_ns[1] = (int64_t)t1.tv_sec * 1000000000 + t1.tv_nsec;
  return e;
}

hipError_t fused_mlp_persistent(const FusedMlpArgs& a, const PersistArgs& p, hipStream_t s) {
  if (p.n_steps <= 0) return check_dims(a);
  PersistLaunch L;
  PTDT_HIP_CHECK(fused_mlp_persistent_prepare(a, p, &L));
  return persistent_launch(L, p.n_steps, p.cursor_host_pos, s);
}

bool mlp_mfma_persistent_supported(const FusedMlpArgs& a, const PersistArgs& p) { return mfma_engine(a, p); }

}  // namespace ptdt
