// bf16-operand instantiations of the tensor-parallel toy-MLP engine (mlp_tp_impl.h, BF = true):
// BASELINE.json config 2's "toy MLP bf16" DDP step with torch.autocast(bfloat16) rounding points,
// fp32 master weights / momentum / SGD, every product on v_mfma_f32_16x16x32_bf16 or
// v_mfma_f32_16x16x16_bf16 (reference training step: ddp_gpus_torchrun.py:30-35).
#include "mlp_tp_impl.h"

namespace ptdt {
namespace {

template <int LOSS, bool AR, bool VX>
const void* pick_bf(int mt, bool st) {
  if (st)
    return mt == 1 ? (const void*)mlp_tp_kernel<1, LOSS, AR, VX, true, 4, true>
                   : (const void*)mlp_tp_kernel<2, LOSS, AR, VX, true, 4, true>;
  return mt == 1 ? (const void*)mlp_tp_kernel<1, LOSS, AR, VX, false, 4, true>
                 : (const void*)mlp_tp_kernel<2, LOSS, AR, VX, false, 4, true>;
}

template <bool AR, bool VX>
const void* pick_bf_loss(int loss, int mt, bool st) {
  switch (loss) {
    case kLossCEIndex: return pick_bf<kLossCEIndex, AR, VX>(mt, st);
    case kLossMSE: return pick_bf<kLossMSE, AR, VX>(mt, st);
    default: return pick_bf<kLossCESoft, AR, VX>(mt, st);
  }
}

}  // namespace

const void* mlp_tp_bf16_kernel(int loss, bool ar, bool vx, int mt, bool st) {
  return ar ? (vx ? pick_bf_loss<true, true>(loss, mt, st) : pick_bf_loss<true, false>(loss, mt, st))
            : (vx ? pick_bf_loss<false, true>(loss, mt, st) : pick_bf_loss<false, false>(loss, mt, st));
}

}  // namespace ptdt
