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
#include "common.h"
#include "kernels.h"
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

__host__ __device__ __forceinline__ int al4(int n) { return (n + 3) & ~3; }

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
  for (int e = tid; e < d.B * d.Din; e += NT) {
    const int b = e / d.Din, k = e - b * d.Din;
    s.xs[e] = a.X[(int64_t)sel[b] * d.Din + k];
  }
  if constexpr (LOSS != kLossCEIndex) {
    for (int e = tid; e < d.B * d.Dout; e += NT) {
      const int b = e / d.Dout, c = e - b * d.Dout;
      s.ys[e] = a.Yf[(int64_t)sel[b] * d.Dout + c];
    }
  } else {
    int* yl = reinterpret_cast<int*>(s.ys);
    for (int b = tid; b < d.B; b += NT) yl[b] = (int)a.Yi[sel[b]];
  }
}

// forward + loss + backward of one batch staged in LDS. Gradients (times
// grad_scale / loss denominator) go to gdst (accumulated when acc); the mean
// loss to *loss_out (thread 0). Ends with every gdst write issued (no barrier).
template <bool HID, int LOSS>
__device__ __forceinline__ void step_body(const FusedMlpArgs& a, const Dims& d, const float* Ps, const Scratch& s,
                                          float* gdst, bool acc, float* loss_out, int tid, int NT) {
  const int B = d.B, Din = d.Din, H = d.H, Dout = d.Dout, Dh = d.Dh;
  const float* W1 = Ps;
  const float* b1 = Ps + d.nW1;
  const float* W2 = Ps + d.nW1 + d.nb1;
  const float* b2 = W2 + d.nW2;
  float *as = s.as, *zs = s.zs, *ds = s.ds;
  const float* xs = s.xs;
  const float* ys = s.ys;

  if constexpr (HID) {
    const bool v_in = (Din & 3) == 0;
    for (int e = tid; e < B * H; e += NT) {
      const int b = e / H, j = e - b * H;
      const float v = (d.nb1 ? b1[j] : 0.f) + dot_lds(xs + b * Din, W1 + j * Din, Din, v_in);
      as[e] = fmaxf(v, 0.f);
    }
    __syncthreads();
  }
  const float* act = HID ? as : xs;
  const bool v_out = (Dh & 3) == 0 && ((d.nW1 + d.nb1) & 3) == 0;
  for (int e = tid; e < B * Dout; e += NT) {
    const int b = e / Dout, c = e - b * Dout;
    zs[e] = (d.nb2 ? b2[c] : 0.f) + dot_lds(act + b * Dh, W2 + c * Dh, Dh, v_out);
  }
  __syncthreads();

  // loss + dL/dlogits (unnormalised; 1/denominator folded into coef)
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
      cnt += (float)Dout;
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
        cnt += 1.f;
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
  lsum = block_sum(lsum, s.red);
  cnt = block_sum(cnt, s.red + 16);
  const float denom = cnt > 0.f ? cnt : 1.f;
  if (tid == 0) *loss_out = (cnt > 0.f) ? lsum / denom : (LOSS == kLossCEIndex ? NAN : 0.f);
  const float coef = a.grad_scale / denom;
  __syncthreads();

  float* gW1 = gdst;
  float* gb1 = gdst + d.nW1;
  float* gW2 = gdst + d.nW1 + d.nb1;
  float* gb2 = gW2 + d.nW2;
  for (int e = tid; e < d.nW2 + d.nb2; e += NT) {
    float sm = 0.f;
    if (e < d.nW2) {
      const int c = e / Dh, j = e - c * Dh;
      for (int b = 0; b < B; ++b) sm = fmaf(zs[b * Dout + c], act[b * Dh + j], sm);
      sm *= coef;
      gW2[e] = acc ? gW2[e] + sm : sm;
    } else {
      const int c = e - d.nW2;
      for (int b = 0; b < B; ++b) sm += zs[b * Dout + c];
      sm *= coef;
      gb2[c] = acc ? gb2[c] + sm : sm;
    }
  }
  if constexpr (HID) {
    for (int e = tid; e < B * H; e += NT) {
      const int b = e / H, j = e - b * H;
      float sm = 0.f;
      if (as[e] > 0.f)
        for (int c = 0; c < Dout; ++c) sm = fmaf(zs[b * Dout + c], W2[c * H + j], sm);
      ds[e] = sm;
    }
    __syncthreads();
    for (int e = tid; e < d.nW1 + d.nb1; e += NT) {
      float sm = 0.f;
      if (e < d.nW1) {
        const int j = e / Din, k = e - j * Din;
        for (int b = 0; b < B; ++b) sm = fmaf(ds[b * H + j], xs[b * Din + k], sm);
        sm *= coef;
        gW1[e] = acc ? gW1[e] + sm : sm;
      } else {
        const int j = e - d.nW1;
        for (int b = 0; b < B; ++b) sm += ds[b * H + j];
        sm *= coef;
        gb1[j] = acc ? gb1[j] + sm : sm;
      }
    }
  }
}

// Average `np` gradients held in LDS across ranks (in place). world == 1 is
// the identity: DDP over one rank averages nothing.
__device__ __forceinline__ void allreduce_lds(const XgmiArgs& ar, uint32_t seq, float* gs, float* tmp, int np,
                                              int tid, int NT, int* lds_flag = nullptr) {
  if (ar.world <= 1) return;
  xgmi_push(ar, seq, gs, np, tid, NT);
  xgmi_gather_lds(ar, seq, 0, np, tmp, tid, NT, lds_flag);
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
  if constexpr (AR) ar_seq = *a.ar.seq + 1u;

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

  step_body<HID, LOSS>(a, d, Ps, s, AR ? gs : a.G, !AR && a.accumulate != 0, a.loss_out, tid, NT);

  if constexpr (AR) {
    __syncthreads();
    allreduce_lds(a.ar, ar_seq, gs, tmp, np, tid, NT);
    for (int i = tid; i < np; i += NT) {
      const float g = gs[i];
      a.G[i] = g;  // .grad holds the global average, as after DDP's finalize
      if constexpr (MODE == kArPost)
        a.P[i] = sgd_one(Ps[i], g, a.mom, i, first, a.lr, a.momentum, a.dampening, a.weight_decay, a.nesterov);
    }
    if (tid == 0) {
      if (a.ar.world > 1) *a.ar.seq = ar_seq;
      if (MODE == kArPost && a.opt_step != nullptr) *a.opt_step += 1;
    }
  }
}

// ------------------------------------------------------------------ persistent engine
template <bool HID, int LOSS>
__global__ void __launch_bounds__(1024) fused_mlp_persistent_kernel(FusedMlpArgs a, PersistArgs pa) {
  extern __shared__ float lds[];
  constexpr bool FY = LOSS != kLossCEIndex;
  const int tid = threadIdx.x, NT = blockDim.x;
  const Dims full(a.B, a.Din, HID ? a.H : 0, a.Dout, a.has_bias != 0);
  const int np = full.np, B = full.B;
  const bool use_mom = a.mom != nullptr && a.momentum != 0.f;

  float* Ps = lds;                                 // live parameters
  float* Ms = Ps + al4(np);                        // live momentum
  float* gs = Ms + al4(np);                        // grads of the current step
  Scratch s;
  s.xs = gs + al4(np);
  s.as = s.xs + al4(B * full.Din);
  s.zs = s.as + al4(B * full.H);
  s.ds = s.zs + al4(B * full.Dout);
  s.ys = s.ds + al4(B * full.H);
  s.red = s.ys + al4(FY ? B * full.Dout : B);
  float* tmp = s.red + 32;                         // [world * np]
  int* eidx = reinterpret_cast<int*>(tmp + al4((a.ar.world > 1 ? a.ar.world : 1) * np));  // [num_samples]
  int* lds_err = eidx + al4(pa.num_samples);       // set by a timed-out poll
  if (tid == 0) *lds_err = 0;

  // ---- load resident state
  for (int i = tid; i < np; i += NT) {
    Ps[i] = a.P[i];
    Ms[i] = use_mom ? a.mom[i] : 0.f;
  }
  int epoch = pa.cursor[0], j = pa.cursor[1];
  const int steps_per_epoch = (pa.num_samples + B - 1) / B;
  int opt_step = a.opt_step ? *a.opt_step : 0;
  uint32_t seq = a.ar.world > 1 ? *a.ar.seq : 0u;
  if (j != 0) rank_epoch_indices(eidx, (uint32_t)pa.N, pa.W, pa.rank, pa.num_samples, pa.seed, epoch, pa.shuffle,
                                 tid, NT);
  __syncthreads();

  for (int step = 0; step < pa.n_steps; ++step) {
    if (j == 0) {  // new epoch: this rank's DistributedSampler shard, computed in place
      rank_epoch_indices(eidx, (uint32_t)pa.N, pa.W, pa.rank, pa.num_samples, pa.seed, epoch, pa.shuffle, tid, NT);
      __syncthreads();
    }
    const int b0 = j * B;
    const int bsz = pa.num_samples - b0 < B ? pa.num_samples - b0 : B;
    const Dims d(bsz, full.Din, full.H, full.Dout, a.has_bias != 0);
    gather_batch<LOSS>(a, d, eidx + b0, s, tid, NT);
    __syncthreads();
    step_body<HID, LOSS>(a, d, Ps, s, gs, false, pa.losses + step, tid, NT);
    __syncthreads();
    seq += 1u;
    allreduce_lds(a.ar, seq, gs, tmp, np, tid, NT, lds_err);
    const bool first = opt_step == 0;
    for (int i = tid; i < np; i += NT)
      Ps[i] = sgd_one(Ps[i], gs[i], use_mom ? Ms : nullptr, i, first, a.lr, a.momentum, a.dampening,
                      a.weight_decay, a.nesterov);
    ++opt_step;
    if (++j == steps_per_epoch) {
      j = 0;
      ++epoch;
    }
    __syncthreads();
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

template <bool HID>
const void* pick_persist(int loss) {
  switch (loss) {
    case kLossCEIndex: return (const void*)fused_mlp_persistent_kernel<HID, kLossCEIndex>;
    case kLossMSE: return (const void*)fused_mlp_persistent_kernel<HID, kLossMSE>;
    default: return (const void*)fused_mlp_persistent_kernel<HID, kLossCESoft>;
  }
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
  const int64_t fl = 3 * (int64_t)al4(np) + al4(B * Din) + 2 * al4(B * H) + 2 * al4(B * Dout) + al4(B) + 32 +
                     al4((world > 1 ? world : 1) * np) + al4(num_samples) + 4;
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

hipError_t fused_mlp_persistent(const FusedMlpArgs& a, const PersistArgs& p, hipStream_t s) {
  PTDT_HIP_CHECK(check_dims(a));
  if (p.n_steps <= 0) return hipSuccess;
  if (a.update_mode != 2 || a.accumulate || p.cursor == nullptr || p.losses == nullptr || p.num_samples <= 0 ||
      p.N <= 0 || p.W <= 0 || p.rank < 0 || p.rank >= p.W)
    return hipErrorInvalidValue;
  if (a.ar.world > 1 && (num_params(a) > a.ar.max_elems || a.ar.world != p.W || a.ar.rank != p.rank))
    return hipErrorInvalidValue;
  const size_t lds = fused_mlp_persistent_lds_bytes(a.B, a.Din, a.H, a.Dout, p.num_samples, a.ar.world);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const void* fn = a.H > 0 ? pick_persist<true>(a.loss_kind) : pick_persist<false>(a.loss_kind);
  if (lds > 64 * 1024)
    PTDT_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int threads = a.H > 0 ? 1024 : 256;
  void* args[] = {const_cast<FusedMlpArgs*>(&a), const_cast<PersistArgs*>(&p)};
  return hipLaunchKernel(fn, dim3(1), dim3(threads), args, lds, s);
}

}  // namespace ptdt
