// Host dispatch of the single-wave persistent engine (linear_wave_impl.h).
#include "common.h"
#include "kernels.h"

namespace ptdt {

const void* linear_wave_pick_ce_soft(int L, int kp, int dout, bool ar);
const void* linear_wave_pick_ce_index(int L, int kp, int dout, bool ar);
const void* linear_wave_pick_mse(int L, int kp, int dout, bool ar);

namespace {

constexpr int kThreads = 256;  // wave 0 trains, waves 1-3 build index lists

size_t lds_bytes(const PersistArgs& p) {  // two epoch index lists + 8 phase-timer slots
  return (size_t)2 * al4(p.num_samples) * sizeof(int) + 8 * sizeof(unsigned long long);
}

int lanes_per_row(int B) {
  int rows = 1;
  while (rows < B) rows <<= 1;
  return 64 / rows;
}

int pick_kp_value(int Din, int L) {
  const int need = (Din + L - 1) / L;
  for (int kp : {4, 8, 10, 16})
    if (kp >= need) return kp;
  return -1;
}

const void* linear_wave_fn(const FusedMlpArgs& a, const PersistArgs& p) {
  if (a.H != 0 || a.B <= 0 || a.B > 64 || a.Dout <= 0) return nullptr;
  if (a.ar.world > kXgmiMaxRanks) return nullptr;
  if (lds_bytes(p) > 160 * 1024) return nullptr;
  const int L = lanes_per_row(a.B);
  if (L > 8) return nullptr;
  const int kp = pick_kp_value(a.Din, L);
  if (kp < 0) return nullptr;
  const bool ar = a.ar.world > 1;
  switch (a.loss_kind) {
    case kLossCEIndex: return linear_wave_pick_ce_index(L, kp, a.Dout, ar);
    case kLossMSE: return linear_wave_pick_mse(L, kp, a.Dout, ar);
    default: return linear_wave_pick_ce_soft(L, kp, a.Dout, ar);
  }
}

}  // namespace
bool linear_wave_supported(const FusedMlpArgs& a, const PersistArgs& p) { return linear_wave_fn(a, p) != nullptr; }

hipError_t linear_wave_persistent(const FusedMlpArgs& a, const PersistArgs& p, hipStream_t s) {
  const void* fn = linear_wave_fn(a, p);
  if (fn == nullptr) return hipErrorInvalidValue;
  const size_t lds = lds_bytes(p);
  if (lds > 64 * 1024)
    PTDT_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  void* args[] = {const_cast<FusedMlpArgs*>(&a), const_cast<PersistArgs*>(&p)};
  return hipLaunchKernel(fn, dim3(1), dim3(kThreads), args, lds, s);
}

}  // namespace ptdt
