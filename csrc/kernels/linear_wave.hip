// Host dispatch of the single-wave persistent engine (linear_wave_impl.h).
#include <algorithm>
#include "common.h"
#include "kernels.h"

namespace ptdt {

#define PTDT_LW_DECL(tag) const void* linear_wave_pick_##tag(int L, int R, int kp, int dout);
PTDT_LW_DECL(ce_soft) PTDT_LW_DECL(ce_soft_ar) PTDT_LW_DECL(ce_index) PTDT_LW_DECL(ce_index_ar)
PTDT_LW_DECL(mse) PTDT_LW_DECL(mse_ar)
#undef PTDT_LW_DECL

namespace {

constexpr int kThreads = 256;  // wave 0 trains, waves 1-3 build index lists

size_t lds_bytes(const FusedMlpArgs& a, const PersistArgs& p) {  // two epoch index lists + 8 phase-timer slots
  return (size_t)2 * wave_list_stride(p.num_samples, a.B) * sizeof(int) + 8 * sizeof(unsigned long long);
}
constexpr size_t kStaticLds = 512;  // layout F's static pair-exchange scratch (linear_wave_impl.h)
// loss ring of layout F: (2 epochs + prefetch depth) steps x 64 lane shares
size_t ring_bytes(const FusedMlpArgs& a, const PersistArgs& p) {
  const int S = (p.num_samples + a.B - 1) / a.B;
  return (size_t)(2 * S + kWavePrefetch) * 64 * sizeof(float);
}

const void* pick(int loss, bool ar, int L, int R, int kp, int dout) {
  switch (loss) {
    case kLossCEIndex: return ar ? linear_wave_pick_ce_index_ar(L, R, kp, dout) : linear_wave_pick_ce_index(L, R, kp, dout);
    case kLossMSE: return ar ? linear_wave_pick_mse_ar(L, R, kp, dout) : linear_wave_pick_mse(L, R, kp, dout);
    default: return ar ? linear_wave_pick_ce_soft_ar(L, R, kp, dout) : linear_wave_pick_ce_soft(L, R, kp, dout);
  }
}

int log2i(int v) {
  int r = 0;
  while ((1 << r) < v) ++r;
  return r;
}

// Cycle model of one step on one wave, from tools/microbench_isa.hip issue costs
// (FMA ~5, DPP add ~5.6, permlane swap + add ~30 cycles, a row's CE ~70): picks
// the lane layout (L lanes per row, R rows per lane group) for a shape.
double model_cycles(int L, int R, int kp, int dout) {
  if (L == 0) {  // layout F: features across DPP rows, rows across the 16 lanes of a DPP row
    const bool scatter = dout == 1 && R > 1;
    const double fwd = R * kp * dout * 5.0 + (scatter ? (R == 2 ? 2 : 3) * 25.0 : R * dout * 2 * 30.0);
    const double loss = (scatter ? 1 : R) * (30.0 + 40.0 * dout) + (scatter ? (R == 2 ? 1 : 3) * 25.0 : 0.0);
    const double bwd = R * kp * dout * 5.0 + (kp + 1) * dout * 4 * 5.6;
    return fwd + loss + bwd + (kp + 1) * dout * 10.0 + R * kp * 3.0;
  }
  const bool split = R > 1 && (L == 2 || L == 4) && R <= L;
  const int loss_rows = split ? 1 : R;
  const double fwd = R * kp * dout * 5.0 + R * dout * log2i(L) * 5.6;
  const double loss = loss_rows * (30.0 + 40.0 * dout) + (split ? R * dout * 5.6 : 0.0);
  const double bwd = R * kp * dout * 5.0 + (kp + 1) * dout * ((L <= 16 ? log2i(16 / L) : 0) * 5.6 + 2 * 30.0);
  const double sgd = (kp + 1) * dout * 10.0;
  const double fetch = R * kp * 3.0;
  return fwd + loss + bwd + sgd + fetch;
}

struct Choice {
  const void* fn = nullptr;
  int L = 0, R = 0, kp = 0;
};

Choice choose(const FusedMlpArgs& a, const PersistArgs& p) {
  Choice best;
  if (a.H != 0 || a.B <= 0 || a.B > 64 || a.Dout <= 0) return best;
  if (a.ar.world > kXgmiMaxRanks) return best;
  if (a.B <= 0 || lds_bytes(a, p) + kStaticLds > 160 * 1024) return best;
  const bool ar = a.ar.world > 1;
  static const int kLR[][2] = {{1, 1}, {2, 1}, {4, 1}, {8, 1}, {2, 2}, {4, 2}, {0, 1}, {0, 2}, {0, 4}};
  double best_cost = 1e30;
  const int ldx = a.ldx > 0 ? a.ldx : a.Din;
  for (const auto& lr : kLR) {
    const int L = lr[0], R = lr[1];
    if ((p.variant == kPersistWaveRows && L == 0) || (p.variant == kPersistWaveF && L != 0)) continue;
    const int lanes = L == 0 ? 4 : L;            // feature chunks per row
    const int groups = L == 0 ? 16 : 64 / L;     // row slots
    if (groups * R < a.B) continue;              // rows must fit one pass
    if (ar && groups < a.ar.world) continue;     // one row slot per rank
    const int need = (a.Din + lanes - 1) / lanes;
    int kp = -1;
    for (int c : {4, 5, 8, 10, 16})
      if (c >= need && (lanes * c == a.Din || (a.x_padded && lanes * c <= ldx))) {  // chunks read zero padding
        kp = c;
        break;
      }
    if (kp < 0) continue;
    // layout F gathers through buffer resources: 32-bit byte offsets, 24-bit row index x row bytes
    // (a query with kWaveLdxAny: the caller pads X rows to exactly the layout's width)
    const int64_t row = a.ldx == kWaveLdxAny ? std::max(a.Din, lanes * kp) : ldx;
    if (L == 0 && ((int64_t)p.N * row * 4 >= (1ll << 31) || p.N >= (1 << 24) || row * 4 >= (1 << 24) ||
                   (int64_t)p.N * 8 >= (1ll << 31) || (int64_t)p.N * a.Dout * 4 >= (1ll << 31)))
      continue;
    const void* fn = pick(a.loss_kind, ar, L, R, kp, a.Dout);
    if (fn == nullptr) continue;
    const double cost = model_cycles(L, R, kp, a.Dout);
    if (cost < best_cost) {
      best_cost = cost;
      best.fn = fn;
      best.L = L;
      best.R = R;
      best.kp = kp;
    }
  }
  return best;
}

}  // namespace
bool linear_wave_supported(const FusedMlpArgs& a, const PersistArgs& p) { return choose(a, p).fn != nullptr; }

void linear_wave_layout(const FusedMlpArgs& a, const PersistArgs& p, int* L, int* R, int* kp) {
  const Choice c = choose(a, p);
  *L = c.L;
  *R = c.R;
  *kp = c.kp;
}

hipError_t linear_wave_prepare(const FusedMlpArgs& a, const PersistArgs& p, PersistLaunch* out) {
  const Choice c = choose(a, p);
  if (c.fn == nullptr) return hipErrorInvalidValue;
  out->fn = c.fn;
  out->threads = kThreads;
  out->a = a;
  out->p = p;
  out->p.loss_ring = 0;
  out->lds = lds_bytes(a, p);
  if (c.L == 0 && out->lds + ring_bytes(a, p) + kStaticLds <= 160 * 1024) {
    out->p.loss_ring = 1;
    out->lds += ring_bytes(a, p);
  }
  if (out->lds > 64 * 1024)
    PTDT_HIP_CHECK(hipFuncSetAttribute(c.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)out->lds));
  return hipSuccess;
}

hipError_t linear_wave_persistent(const FusedMlpArgs& a, const PersistArgs& p, hipStream_t s) {
  PersistLaunch L;
  PTDT_HIP_CHECK(linear_wave_prepare(a, p, &L));
  return persistent_launch(L, p.n_steps, p.cursor_host_pos, s);
}

}  // namespace ptdt
