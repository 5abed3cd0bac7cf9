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

constexpr int kThreads = 256;

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

__global__ void __launch_bounds__(kThreads) fused_mlp_step_kernel(FusedMlpArgs a) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x;
  const int B = a.B, Din = a.Din, H = a.H, Dout = a.Dout;
  const int Dh = H > 0 ? H : Din;                 // width feeding the output layer
  const int64_t nW1 = H > 0 ? (int64_t)H * Din : 0;
  const int64_t nb1 = (H > 0 && a.has_bias) ? H : 0;
  const int64_t nW2 = (int64_t)Dout * Dh;
  const int64_t nb2 = a.has_bias ? Dout : 0;
  const int64_t np = nW1 + nb1 + nW2 + nb2;

  float* Ps = lds;                    // [np]
  float* xs = Ps + np;                // [B*Din]
  float* as = xs + (int64_t)B * Din;  // [B*H]
  float* zs = as + (int64_t)B * H;    // [B*Dout]  logits -> dlogits
  float* ds = zs + (int64_t)B * Dout; // [B*H]     d(pre-activation)
  float* red = ds + (int64_t)B * H;   // [16]

  // ---- 1. deferred optimizer step of the previous iteration + param staging
  if (a.pre_lr > 0.f) {
    const bool first = (a.opt_step != nullptr) ? (*a.opt_step == 0) : false;
    for (int64_t i = tid; i < np; i += kThreads) {
      float p = sgd_one(a.P[i], a.G[i], a.mom, i, first, a.pre_lr, a.pre_momentum,
                        a.pre_dampening, a.pre_weight_decay, a.pre_nesterov);
      a.P[i] = p;
      Ps[i] = p;
    }
    __syncthreads();
    if (tid == 0 && a.opt_step != nullptr) *a.opt_step += 1;
  } else {
    for (int64_t i = tid; i < np; i += kThreads) Ps[i] = a.P[i];
  }
  const float* W1 = Ps;
  const float* b1 = Ps + nW1;
  const float* W2 = Ps + nW1 + nb1;
  const float* b2 = W2 + nW2;

  // ---- 2. batch gather (sampler indices -> rows of the resident dataset)
  for (int64_t e = tid; e < (int64_t)B * Din; e += kThreads) {
    const int b = (int)(e / Din), k = (int)(e % Din);
    const int64_t row = a.idx ? (int64_t)a.idx[b] : b;
    xs[e] = a.X[row * Din + k];
  }
  __syncthreads();

  // ---- 3. forward
  if (H > 0) {
    for (int64_t e = tid; e < (int64_t)B * H; e += kThreads) {
      const int b = (int)(e / H), j = (int)(e % H);
      float acc = nb1 ? b1[j] : 0.f;
      const float* xr = xs + (int64_t)b * Din;
      const float* wr = W1 + (int64_t)j * Din;
      for (int k = 0; k < Din; ++k) acc = fmaf(xr[k], wr[k], acc);
      as[e] = fmaxf(acc, 0.f);
    }
    __syncthreads();
  }
  const float* act = H > 0 ? as : xs;
  for (int64_t e = tid; e < (int64_t)B * Dout; e += kThreads) {
    const int b = (int)(e / Dout), c = (int)(e % Dout);
    float acc = nb2 ? b2[c] : 0.f;
    const float* ar = act + (int64_t)b * Dh;
    const float* wr = W2 + (int64_t)c * Dh;
    for (int j = 0; j < Dh; ++j) acc = fmaf(ar[j], wr[j], acc);
    zs[e] = acc;
  }
  __syncthreads();

  // ---- 4. loss + dL/dlogits (unnormalised; 1/denominator folded into coef)
  float lsum = 0.f, cnt = 0.f;
  for (int b = tid; b < B; b += kThreads) {
    float* z = zs + (int64_t)b * Dout;
    const int64_t row = a.idx ? (int64_t)a.idx[b] : b;
    if (a.loss_kind == kLossMSE) {
      const float* t = a.Yf + row * Dout;
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
      const float* t = a.Yf + row * Dout;
      float tsum = 0.f, l = 0.f;
      for (int c = 0; c < Dout; ++c) {
        tsum += t[c];
        l -= t[c] * (z[c] - lse);
      }
      for (int c = 0; c < Dout; ++c) z[c] = expf(z[c] - lse) * tsum - t[c];
      lsum += l;
      cnt += 1.f;
    } else {  // class index
      const int64_t y = a.Yi[row];
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
  cnt = block_sum(cnt, red + 8);
  const float denom = cnt > 0.f ? cnt : 1.f;
  if (tid == 0) *a.loss_out = (cnt > 0.f) ? lsum / denom : (a.loss_kind == kLossCEIndex ? NAN : 0.f);
  const float coef = a.grad_scale / denom;
  __syncthreads();

  // ---- 5. backward, gradients straight into the bucket
  float* gW1 = a.G;
  float* gb1 = a.G + nW1;
  float* gW2 = a.G + nW1 + nb1;
  float* gb2 = gW2 + nW2;
  const bool acc = a.accumulate != 0;
  for (int64_t e = tid; e < nW2 + nb2; e += kThreads) {
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
    for (int64_t e = tid; e < (int64_t)B * H; e += kThreads) {
      const int b = (int)(e / H), j = (int)(e % H);
      float s = 0.f;
      if (as[e] > 0.f)
        for (int c = 0; c < Dout; ++c) s = fmaf(zs[(int64_t)b * Dout + c], W2[(int64_t)c * H + j], s);
      ds[e] = s;
    }
    __syncthreads();
    for (int64_t e = tid; e < nW1 + nb1; e += kThreads) {
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
}

}  // namespace

size_t fused_mlp_lds_bytes(int B, int Din, int H, int Dout) {
  const int64_t Dh = H > 0 ? H : Din;
  const int64_t np = (H > 0 ? (int64_t)H * Din + H : 0) + (int64_t)Dout * Dh + Dout;
  const int64_t fl = np + (int64_t)B * Din + 2 * (int64_t)B * H + (int64_t)B * Dout + 16;
  return (size_t)fl * sizeof(float);
}

hipError_t fused_mlp_step(const FusedMlpArgs& a, hipStream_t s) {
  const size_t lds = fused_mlp_lds_bytes(a.B, a.Din, a.H, a.Dout);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  if (a.B <= 0 || a.Din <= 0 || a.Dout <= 0 || a.H < 0) return hipErrorInvalidValue;
  if (lds > 64 * 1024) {
    PTDT_HIP_CHECK(hipFuncSetAttribute((const void*)fused_mlp_step_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  }
  hipLaunchKernelGGL(fused_mlp_step_kernel, dim3(1), dim3(kThreads), lds, s, a);
  return hipGetLastError();
}

}  // namespace ptdt
