// Fused per-rank train step of a small Linear[-ReLU-Linear] model in ONE launch.
//
// Replaces, for the DDP toy workloads, the ~10 tiny ATen launches of the
// reference step (ddp_gpus.py:34-39: zero_grad, addmm, cross_entropy fwd,
// fill, cross_entropy bwd, addmm bwd, DDP bucket copy+scale, foreach SGD) plus
// its per-step H2D copies (ddp_gpus.py:47-48) with:
//   * an on-device gather of the batch from the resident dataset by sampler
//     indices (no DataLoader, no H2D per step),
//   * forward, loss, backward entirely in LDS,
//   * gradients written already scaled by 1/world_size into the flat DDP bucket
//     (the bucket IS the .grad storage, no pack/unpack),
//   * the previous step's SGD update applied first from the all-reduced bucket
//     (deferred update) so the optimizer costs no launch of its own.
// At these sizes (B=32, Din=20) the step is pure latency: one workgroup, all
// operands in LDS, no MFMA (a 32x1x20 product cannot fill a 16x16x32 tile).
#include "common.h"
#include "kernels.h"

namespace ptdt {
namespace {

__device__ __forceinline__ float sgd_one(float p, float g, float* mom, int64_t i, bool first,
                                         float lr, float mu, float damp, float wd, int nesterov) {
  float d = g + wd * p;
  if (mom != nullptr && mu != 0.f) {
    float buf = first ? d : mu * mom[i] + (1.f - damp) * d;
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

// Critical path = two dependent global round trips: (sampler indices || params,
// grads, opt state) -> barrier -> (dataset rows X, Y gathered by index) ->
// barrier; everything after runs out of LDS. blockDim.x is 256 for the
// reference's single Linear, 1024 (16 waves) when a hidden layer gives enough
// independent work to hide LDS latency.
__global__ void __launch_bounds__(1024) fused_mlp_step_kernel(FusedMlpArgs a) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x, NT = blockDim.x;
  const int B = a.B, Din = a.Din, H = a.H, Dout = a.Dout;
  const int Dh = H > 0 ? H : Din;                 // width feeding the output layer
  const int64_t nW1 = H > 0 ? (int64_t)H * Din : 0;
  const int64_t nb1 = (H > 0 && a.has_bias) ? H : 0;
  const int64_t nW2 = (int64_t)Dout * Dh;
  const int64_t nb2 = a.has_bias ? Dout : 0;
  const int64_t np = nW1 + nb1 + nW2 + nb2;
  const bool soft_or_mse = a.loss_kind != kLossCEIndex;

  // LDS carve-up (floats); every array starts 16-B aligned
  auto al4 = [](int64_t n) { return (n + 3) & ~(int64_t)3; };
  float* Ps = lds;                           // [np]
  float* xs = Ps + al4(np);                  // [B*Din]
  float* as = xs + al4((int64_t)B * Din);    // [B*H]
  float* zs = as + al4((int64_t)B * H);      // [B*Dout]  logits -> dlogits
  float* ds = zs + al4((int64_t)B * Dout);   // [B*H]     d(pre-activation)
  float* ys = ds + al4((int64_t)B * H);      // [B*Dout] float targets, or [B] labels (as int)
  int* sidx = reinterpret_cast<int*>(ys + al4((int64_t)B * (soft_or_mse ? Dout : 1)));  // [B]
  float* red = reinterpret_cast<float*>(sidx + al4(B));  // [32]
  float* gs = red + 32;                      // [np] local grads (in-kernel all-reduce only)
  const bool use_ar = a.ar.world > 0;
  const uint32_t ar_seq = use_ar ? *a.ar.seq + 1u : 0u;
  const bool step_first = (a.opt_step != nullptr) ? (*a.opt_step == 0) : false;

  // ---- trip 1: sampler indices, and the deferred optimizer step of the previous iteration
  for (int b = tid; b < B; b += NT) sidx[b] = a.idx ? a.idx[b] : b;
  const bool pre = a.update_mode == 1 && a.lr > 0.f;
  if (pre) {
    for (int64_t i = tid; i < np; i += NT) {
      const float p = sgd_one(a.P[i], a.G[i], a.mom, i, step_first, a.lr, a.momentum, a.dampening,
                              a.weight_decay, a.nesterov);
      a.P[i] = p;
      Ps[i] = p;
    }
  } else {
    for (int64_t i = tid; i < np; i += NT) Ps[i] = a.P[i];
  }
  __syncthreads();
  if (pre && tid == 0 && a.opt_step != nullptr) *a.opt_step += 1;
  const float* W1 = Ps;
  const float* b1 = Ps + nW1;
  const float* W2 = Ps + nW1 + nb1;
  const float* b2 = W2 + nW2;

  // ---- trip 2: gather the batch rows (features and targets) into LDS
  for (int64_t e = tid; e < (int64_t)B * Din; e += NT) {
    const int b = (int)(e / Din), k = (int)(e % Din);
    xs[e] = a.X[(int64_t)sidx[b] * Din + k];
  }
  if (soft_or_mse) {
    for (int64_t e = tid; e < (int64_t)B * Dout; e += NT) {
      const int b = (int)(e / Dout), c = (int)(e % Dout);
      ys[e] = a.Yf[(int64_t)sidx[b] * Dout + c];
    }
  } else {
    int* yl = reinterpret_cast<int*>(ys);
    for (int b = tid; b < B; b += NT) yl[b] = (int)a.Yi[sidx[b]];
  }
  __syncthreads();

  // ---- forward
  const bool v_in = (Din & 3) == 0 && ((nW1 + 0) & 3) == 0;
  if (H > 0) {
    for (int64_t e = tid; e < (int64_t)B * H; e += NT) {
      const int b = (int)(e / H), j = (int)(e % H);
      const float acc = (nb1 ? b1[j] : 0.f) + dot_lds(xs + (int64_t)b * Din, W1 + (int64_t)j * Din, Din, v_in);
      as[e] = fmaxf(acc, 0.f);
    }
    __syncthreads();
  }
  const float* act = H > 0 ? as : xs;
  const bool v_out = (Dh & 3) == 0 && ((nW1 + nb1) & 3) == 0;
  for (int64_t e = tid; e < (int64_t)B * Dout; e += NT) {
    const int b = (int)(e / Dout), c = (int)(e % Dout);
    zs[e] = (nb2 ? b2[c] : 0.f) + dot_lds(act + (int64_t)b * Dh, W2 + (int64_t)c * Dh, Dh, v_out);
  }
  __syncthreads();

  // ---- loss + dL/dlogits (unnormalised; 1/denominator folded into coef)
  float lsum = 0.f, cnt = 0.f;
  for (int b = tid; b < B; b += NT) {
    float* z = zs + (int64_t)b * Dout;
    if (a.loss_kind == kLossMSE) {
      const float* t = ys + (int64_t)b * Dout;
      for (int c = 0; c < Dout; ++c) {
        const float d = z[c] - t[c];
        lsum = fmaf(d, d, lsum);
        z[c] = 2.f * d;
      }
      cnt += (float)Dout;
      continue;
    }
    float m = -INFINITY;
    for (int c = 0; c < Dout; ++c) m = fmaxf(m, z[c]);
    float se = 0.f;
    for (int c = 0; c < Dout; ++c) se += expf(z[c] - m);
    const float lse = m + logf(se);
    if (a.loss_kind == kLossCESoft) {
      const float* t = ys + (int64_t)b * Dout;
      float tsum = 0.f, l = 0.f;
      for (int c = 0; c < Dout; ++c) {
        tsum += t[c];
        l -= t[c] * (z[c] - lse);
      }
      for (int c = 0; c < Dout; ++c) z[c] = expf(z[c] - lse) * tsum - t[c];
      lsum += l;
      cnt += 1.f;
    } else {  // class index
      const int y = reinterpret_cast<const int*>(ys)[b];
      if (y == a.ignore_index) {
        for (int c = 0; c < Dout; ++c) z[c] = 0.f;
      } else {
        lsum += lse - z[y];
        for (int c = 0; c < Dout; ++c) z[c] = expf(z[c] - lse) - (c == y ? 1.f : 0.f);
        cnt += 1.f;
      }
    }
  }
  lsum = block_sum(lsum, red);
  cnt = block_sum(cnt, red + 16);
  const float denom = cnt > 0.f ? cnt : 1.f;
  if (tid == 0) *a.loss_out = (cnt > 0.f) ? lsum / denom : (a.loss_kind == kLossCEIndex ? NAN : 0.f);
  const float coef = a.grad_scale / denom;
  __syncthreads();

  // ---- backward, gradients straight into the bucket
  float* gdst = use_ar ? gs : a.G;  // with the in-kernel all-reduce, local grads stay in LDS
  float* gW1 = gdst;
  float* gb1 = gdst + nW1;
  float* gW2 = gdst + nW1 + nb1;
  float* gb2 = gW2 + nW2;
  const bool acc = a.accumulate != 0 && !use_ar;
  for (int64_t e = tid; e < nW2 + nb2; e += NT) {
    float s = 0.f;
    if (e < nW2) {
      const int c = (int)(e / Dh), j = (int)(e % Dh);
      for (int b = 0; b < B; ++b) s = fmaf(zs[(int64_t)b * Dout + c], act[(int64_t)b * Dh + j], s);
      s *= coef;
      gW2[e] = acc ? gW2[e] + s : s;
    } else {
      const int c = (int)(e - nW2);
      for (int b = 0; b < B; ++b) s += zs[(int64_t)b * Dout + c];
      s *= coef;
      gb2[c] = acc ? gb2[c] + s : s;
    }
  }
  if (H > 0) {
    for (int64_t e = tid; e < (int64_t)B * H; e += NT) {
      const int b = (int)(e / H), j = (int)(e % H);
      float s = 0.f;
      if (as[e] > 0.f)
        for (int c = 0; c < Dout; ++c) s = fmaf(zs[(int64_t)b * Dout + c], W2[(int64_t)c * H + j], s);
      ds[e] = s;
    }
    __syncthreads();
    for (int64_t e = tid; e < nW1 + nb1; e += NT) {
      float s = 0.f;
      if (e < nW1) {
        const int j = (int)(e / Din), k = (int)(e % Din);
        for (int b = 0; b < B; ++b) s = fmaf(ds[(int64_t)b * H + j], xs[(int64_t)b * Din + k], s);
        s *= coef;
        gW1[e] = acc ? gW1[e] + s : s;
      } else {
        const int j = (int)(e - nW1);
        for (int b = 0; b < B; ++b) s += ds[(int64_t)b * H + j];
        s *= coef;
        gb1[j] = acc ? gb1[j] + s : s;
      }
    }
  }
  if (!use_ar) return;

  // ---- in-kernel one-shot all-reduce over xGMI, then this step's SGD update
  __syncthreads();
  xgmi_push(a.ar, ar_seq, gs, (int)np, tid, NT);
  const float inv_w = 1.f / (float)a.ar.world;
  const bool post = a.update_mode == 2 && a.lr > 0.f;
  for (int64_t i = tid; i < np; i += NT) {
    const float g = xgmi_gather_sum(a.ar, ar_seq, (int)i) * inv_w;
    a.G[i] = g;  // .grad holds the global average, as after DDP's finalize
    if (post)
      a.P[i] = sgd_one(Ps[i], g, a.mom, i, step_first, a.lr, a.momentum, a.dampening, a.weight_decay,
                       a.nesterov);
  }
  __syncthreads();
  if (tid == 0) {
    *a.ar.seq = ar_seq;
    if (post && a.opt_step != nullptr) *a.opt_step += 1;
  }
}

}  // namespace

size_t fused_mlp_lds_bytes(int B, int Din, int H, int Dout) {
  auto al4 = [](int64_t n) { return (n + 3) & ~(int64_t)3; };
  const int64_t Dh = H > 0 ? H : Din;
  const int64_t np = (H > 0 ? (int64_t)H * Din + H : 0) + (int64_t)Dout * Dh + Dout;
  const int64_t fl = al4(np) + al4((int64_t)B * Din) + 2 * al4((int64_t)B * H) + 2 * al4((int64_t)B * Dout) +
                     al4(B) + al4(B) + 32 + al4(np);
  return (size_t)fl * sizeof(float);
}

hipError_t fused_mlp_step(const FusedMlpArgs& a, hipStream_t s) {
  const size_t lds = fused_mlp_lds_bytes(a.B, a.Din, a.H, a.Dout);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (a.B <= 0 || a.Din <= 0 || a.Dout <= 0 || a.H < 0) return hipErrorInvalidValue;
  if (a.ar.world > 0) {
    const int64_t Dh = a.H > 0 ? a.H : a.Din;
    const int64_t np = (a.H > 0 ? (int64_t)a.H * a.Din + (a.has_bias ? a.H : 0) : 0) + (int64_t)a.Dout * Dh +
                       (a.has_bias ? a.Dout : 0);
    if (np > a.ar.max_elems || a.update_mode == 1 || a.accumulate) return hipErrorInvalidValue;
  }
  if (lds > 64 * 1024) {
    PTDT_HIP_CHECK(hipFuncSetAttribute((const void*)fused_mlp_step_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  }
  const int threads = a.H > 0 ? 1024 : 256;
  hipLaunchKernelGGL(fused_mlp_step_kernel, dim3(1), dim3(threads), lds, s, a);
  return hipGetLastError();
}

}  // namespace ptdt
