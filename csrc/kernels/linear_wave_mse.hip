// Single-wave engine instantiations for one loss (split per loss so the
// instantiation table compiles in parallel). See linear_wave_impl.h.
#include "linear_wave_impl.h"

namespace ptdt {
const void* linear_wave_pick_mse(int L, int kp, int dout, bool ar) { return lw::pick<kLossMSE>(L, kp, dout, ar); }
}  // namespace ptdt
