// Single-wave engine instantiations: ce_index, without the in-kernel all-reduce.
// One translation unit per (loss, all-reduce) so the table compiles in parallel.
// See linear_wave_impl.h.
#include "linear_wave_impl.h"

namespace ptdt {
const void* linear_wave_pick_ce_index(int L, int R, int kp, int dout) {
  return lw::pick<kLossCEIndex, false>(L, R, kp, dout);
}
}  // namespace ptdt
