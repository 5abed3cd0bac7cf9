// Tensor-parallel persistent DDP step engine for Linear(Din,H)-ReLU-Linear(H,Dout):
// the exact-fp32 instantiations and the host side (support check, kernel choice,
// launch plan). The kernel itself is csrc/kernels/mlp_tp_impl.h; the bf16-operand
// instantiations live in mlp_tp_bf16.hip (separate unit: parallel compilation).
#include "mlp_tp_impl.h"

namespace ptdt {
namespace {

// mt 3: two input tiles whose second one holds at most 8 real inputs (Din + bias <= 24): fwd1 runs
// 2 of that tile's 4 K-steps (kernel KL = 2)
template <int LOSS, bool AR, bool VX>
const void* pick_mt(int mt, bool st) {
  if (st)  // phase timers (diagnostic instantiations; the all-reduce's share shows at world > 1)
    return mt == 1 ? (const void*)mlp_tp_kernel<1, LOSS, AR, VX, true>
                   : (mt == 3 ? (const void*)mlp_tp_kernel<2, LOSS, AR, VX, true, 2>
                              : (const void*)mlp_tp_kernel<2, LOSS, AR, VX, true>);
  return mt == 1 ? (const void*)mlp_tp_kernel<1, LOSS, AR, VX, false>
                 : (mt == 3 ? (const void*)mlp_tp_kernel<2, LOSS, AR, VX, false, 2>
                            : (const void*)mlp_tp_kernel<2, LOSS, AR, VX, false>);
}

template <bool AR, bool VX>
const void* pick_loss_tp(int loss, int mt, bool st) {
  switch (loss) {
    case kLossCEIndex: return pick_mt<kLossCEIndex, AR, VX>(mt, st);
    case kLossMSE: return pick_mt<kLossMSE, AR, VX>(mt, st);
    default: return pick_mt<kLossCESoft, AR, VX>(mt, st);
  }
}

bool tp_bf16(const PersistArgs& p) { return p.variant == kPersistTpBf16; }

}  // namespace

bool mlp_tp_supported(const FusedMlpArgs& a, const PersistArgs& p) {
  if (a.H < 16 || a.H > 64 || a.H % 16 != 0) return false;
  if (a.B < 1 || a.B > 32 || a.Din < 1 || a.Din + (a.has_bias ? 1 : 0) > 32 || a.Dout < 1 || a.Dout > 16)
    return false;
  if (a.ar.world > kXgmiMaxRanks) return false;
  // lane-major exchange slots: NW waves x NV values x 64 lanes per rank and parity (max_elems 0:
  // a configuration query without a buffer yet -- XgmiAllReduce's default holds 16x more)
  if (a.ar.world > 1 && a.ar.max_elems > 0 && (a.H / 16) * (4 * tp_mt(a) + 5) * 64 > a.ar.max_elems) return false;
  if (p.N <= 0 || p.num_samples <= 0) return false;
  return tp_lds_bytes(a, p, tp_bf16(p)) <= 160 * 1024;
}

hipError_t mlp_tp_prepare(const FusedMlpArgs& a, const PersistArgs& p, PersistLaunch* out) {
  if (!mlp_tp_supported(a, p)) return hipErrorInvalidValue;
  const bool vx = tp_vec_x(a);
  const bool st = p.stamps != nullptr;
  const bool ar = a.ar.world > 1;
  const void* fn;
  if (tp_bf16(p)) {
    fn = mlp_tp_bf16_kernel(a.loss_kind, ar, vx, tp_mt(a), st);
  } else {
    const int mt = (tp_mt(a) == 2 && a.Din + (a.has_bias ? 1 : 0) <= 24) ? 3 : tp_mt(a);  // 3: pick_mt
    fn = ar ? (vx ? pick_loss_tp<true, true>(a.loss_kind, mt, st) : pick_loss_tp<true, false>(a.loss_kind, mt, st))
            : (vx ? pick_loss_tp<false, true>(a.loss_kind, mt, st) : pick_loss_tp<false, false>(a.loss_kind, mt, st));
  }
  const size_t lds = tp_lds_bytes(a, p, tp_bf16(p));
  if (lds > 64 * 1024) PTDT_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  out->fn = fn;
  out->threads = 64 * (a.H / 16 + 1);  // compute waves + the helper wave
  out->lds = lds;
  out->a = a;
  out->p = p;
  return hipSuccess;
}

}  // namespace ptdt
