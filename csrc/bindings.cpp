// Python bindings of the native layer: gfx950 kernels (csrc/kernels), the RCCL
// communicator (csrc/comm) and the DDP reducer (csrc/reducer).
//
// Every kernel wrapper validates device/dtype/contiguity/shape on the host
// before launching (a bad launch on MI355X can reset the whole node) and
// launches on the caller's current HIP stream, so all of them are capturable
// into hipGraphs via torch.cuda.graph.
#include <time.h>

#include <map>
#include <mutex>
#include <utility>
#include <vector>
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>

#include "comm/rccl_comm.h"
#include "comm/xgmi_comm.h"
#include "kernels/kernels.h"
#include "reducer/reducer.h"

namespace py = pybind11;
using at::Tensor;

namespace ptdt {
namespace {

hipStream_t cur_stream(const Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void hip_check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, " failed: ", hipGetErrorString(e));
}

int dt_of(const Tensor& t) {
  if (t.scalar_type() == at::kFloat) return kF32;
  if (t.scalar_type() == at::kBFloat16) return kBF16;
  TORCH_CHECK(false, "ptdt kernels support float32 and bfloat16, got ", t.scalar_type());
  return -1;
}

// the LLM.int8 pieces also take IEEE half (the reference's load_in_8bit Llama runs in fp16)
int dt_of16(const Tensor& t) {
  if (t.scalar_type() == at::kHalf) return kF16;
  return dt_of(t);
}

at::ScalarType scalar_of(const std::string& name) {
  if (name == "float32") return at::kFloat;
  if (name == "bfloat16") return at::kBFloat16;
  if (name == "float16") return at::kHalf;
  TORCH_CHECK(false, "int8_mm: out dtype must be float32, bfloat16 or float16, got ", name);
  return at::kFloat;
}

void check_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

// Elementwise optimizer operands: any dense memory order (channels_last conv
// weights), as long as every operand of one parameter shares it.
// same element order in memory: equal strides on every dimension of size > 1 (size-1 dimensions
// carry arbitrary strides, e.g. a [C, K, 1, 1] tensor contiguous vs channels_last)
bool same_memory_order(const Tensor& a, const Tensor& b) {
  if (a.sizes() != b.sizes()) return false;
  for (int64_t d = 0; d < a.dim(); ++d)
    if (a.size(d) > 1 && a.stride(d) != b.stride(d)) return false;
  return true;
}

void check_dense_like(const Tensor& p, const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_non_overlapping_and_dense(), name, " must be dense (non-overlapping)");
  TORCH_CHECK(t.numel() == p.numel() &&
                  (t.strides() == p.strides() || (t.is_contiguous() && p.is_contiguous()) || same_memory_order(t, p)),
              name, " must have the parameter's memory layout");
}

template <typename T>
T* ptr_or_null(const c10::optional<Tensor>& t) {
  return (t.has_value() && t->defined()) ? static_cast<T*>(t->data_ptr()) : nullptr;
}

// ------------------------------------------------------------- fused step
void fused_mlp_step_py(Tensor X, c10::optional<Tensor> Yf, c10::optional<Tensor> Yi,
                    c10::optional<Tensor> idx, Tensor P, Tensor G, c10::optional<Tensor> mom,
                    c10::optional<Tensor> opt_step, Tensor loss_out, int64_t B, int64_t Din, int64_t H,
                    int64_t Dout, int64_t loss_kind, int64_t ignore_index, bool has_bias,
                    double grad_scale, bool accumulate, int64_t update_mode, double lr, double momentum,
                    double dampening, double weight_decay, bool nesterov, std::shared_ptr<XgmiComm> ar) {
  check_gpu(X, "X");
  check_gpu(P, "P");
  check_gpu(G, "G");
  TORCH_CHECK(X.scalar_type() == at::kFloat && P.scalar_type() == at::kFloat && G.scalar_type() == at::kFloat,
              "fused_mlp_step: fp32 dataset/params/grads");
  TORCH_CHECK(X.dim() == 2 && X.size(1) == Din, "fused_mlp_step: X must be [N, Din]");
  const int64_t Dh = H > 0 ? H : Din;
  const int64_t np = (H > 0 ? H * Din + (has_bias ? H : 0) : 0) + Dout * Dh + (has_bias ? Dout : 0);
  TORCH_CHECK(P.numel() == np && G.numel() == np, "fused_mlp_step: flat param/grad size mismatch (want ",
              np, ")");
  TORCH_CHECK(loss_out.is_cuda() && loss_out.scalar_type() == at::kFloat && loss_out.numel() >= 1);
  const int64_t N = X.size(0);
  if (idx.has_value() && idx->defined()) {
    check_gpu(*idx, "idx");
    TORCH_CHECK(idx->scalar_type() == at::kInt && idx->numel() >= B, "idx must be int32 with >= B entries");
  } else {
    TORCH_CHECK(B <= N, "fused_mlp_step: B > N without indices");
  }
  if (loss_kind == kLossCEIndex) {
    TORCH_CHECK(Yi.has_value() && Yi->defined() && Yi->scalar_type() == at::kLong && Yi->numel() == N,
                "CE-index needs int64 labels [N]");
    check_gpu(*Yi, "Yi");
  } else {
    TORCH_CHECK(Yf.has_value() && Yf->defined() && Yf->scalar_type() == at::kFloat && Yf->numel() == N * Dout,
                "soft-CE/MSE need float targets [N, Dout]");
    check_gpu(*Yf, "Yf");
  }
  if (mom.has_value() && mom->defined()) TORCH_CHECK(mom->numel() == np && mom->is_cuda());
  TORCH_CHECK(fused_mlp_lds_bytes((int)B, (int)Din, (int)H, (int)Dout) <= 160 * 1024,
              "fused_mlp_step: model/batch too large for one workgroup's LDS; use the layered path");
  c10::hip::HIPGuard guard(X.device().index());
  FusedMlpArgs a{};
  a.X = X.data_ptr<float>();
  a.Yf = ptr_or_null<const float>(Yf);
  a.Yi = ptr_or_null<const int64_t>(Yi);
  a.idx = ptr_or_null<const int32_t>(idx);
  a.P = P.data_ptr<float>();
  a.G = G.data_ptr<float>();
  a.mom = ptr_or_null<float>(mom);
  a.opt_step = ptr_or_null<int32_t>(opt_step);
  a.loss_out = loss_out.data_ptr<float>();
  a.B = (int)B; a.Din = (int)Din; a.H = (int)H; a.Dout = (int)Dout;
  a.loss_kind = (int)loss_kind;
  a.ignore_index = (int)ignore_index;
  a.has_bias = has_bias ? 1 : 0;
  a.grad_scale = (float)grad_scale;
  a.accumulate = accumulate ? 1 : 0;
  a.update_mode = (int)update_mode;
  a.lr = (float)lr;
  a.momentum = (float)momentum;
  a.dampening = (float)dampening;
  a.weight_decay = (float)weight_decay;
  a.nesterov = nesterov ? 1 : 0;
  if (ar) {
    TORCH_CHECK(ar->ready(), "fused_mlp_step: xGMI communicator not opened");
    TORCH_CHECK(np <= ar->max_elems(), "fused_mlp_step: bucket larger than the xGMI buffer");
    TORCH_CHECK(update_mode != 1 && !accumulate, "fused_mlp_step: in-kernel all-reduce needs update_mode 0/2");
    a.ar = ar->args();
  }
  hip_check(ptdt::fused_mlp_step(a, cur_stream(X)), "fused_mlp_step");
}

// Validated persistent-launch arguments (shared by the one-shot call and
// PersistentPlan). Throws on any shape/dtype/sharding mismatch: a bad launch
// of a resident kernel can reset the node.
struct PersistBuild {
  FusedMlpArgs a{};
  PersistArgs pa{};
};

PersistBuild build_persistent(const Tensor& X, const c10::optional<Tensor>& Yf, const c10::optional<Tensor>& Yi,
                              const Tensor& P, const Tensor& G, const c10::optional<Tensor>& mom,
                              const c10::optional<Tensor>& opt_step, int64_t B, int64_t Din, int64_t H, int64_t Dout,
                              int64_t loss_kind, int64_t ignore_index, bool has_bias, double lr, double momentum,
                              double dampening, double weight_decay, bool nesterov,
                              const std::shared_ptr<XgmiComm>& ar, int64_t n_steps, int64_t W, int64_t rank,
                              int64_t num_samples, bool shuffle, int64_t seed, const Tensor& cursor,
                              const Tensor& losses, const c10::optional<Tensor>& stamps, int64_t variant,
                              bool x_zero_padded, const c10::optional<Tensor>& idx, int64_t cursor_j,
                              const c10::optional<Tensor>& lcache = c10::nullopt, int64_t idx_e0 = 0) {
  TORCH_CHECK(X.is_cuda(), "X must be a GPU tensor");  // rows may be padded: checked below
  check_gpu(P, "P");
  check_gpu(G, "G");
  TORCH_CHECK(X.scalar_type() == at::kFloat && P.scalar_type() == at::kFloat && G.scalar_type() == at::kFloat);
  TORCH_CHECK(X.dim() == 2 && X.size(1) == Din && X.stride(1) == 1 && X.stride(0) >= Din,
              "persistent: X must be [N, Din] with unit column stride (rows may be padded)");
  const int64_t N = X.size(0);
  const int64_t Dh = H > 0 ? H : Din;
  const int64_t np = (H > 0 ? H * Din + (has_bias ? H : 0) : 0) + Dout * Dh + (has_bias ? Dout : 0);
  TORCH_CHECK(P.numel() == np && G.numel() == np, "persistent: flat param/grad size mismatch");
  TORCH_CHECK(cursor.is_cuda() && cursor.scalar_type() == at::kInt && cursor.numel() == 2, "cursor: int32[2] GPU");
  TORCH_CHECK(losses.is_cuda() && losses.scalar_type() == at::kFloat && losses.numel() >= n_steps, "losses: f32[n]");
  TORCH_CHECK(num_samples > 0 && num_samples * W >= N && W > 0 && rank >= 0 && rank < W, "persistent: bad sampler");
  if (loss_kind == kLossCEIndex) {
    TORCH_CHECK(Yi.has_value() && Yi->defined() && Yi->scalar_type() == at::kLong && Yi->numel() == N);
  } else {
    TORCH_CHECK(Yf.has_value() && Yf->defined() && Yf->scalar_type() == at::kFloat && Yf->numel() == N * Dout);
  }
  if (mom.has_value() && mom->defined()) TORCH_CHECK(mom->numel() == np && mom->is_cuda());
  const int world = ar ? ar->world() : 1;
  TORCH_CHECK(world == W, "persistent: all-reduce world != sampler world");
  PersistBuild b;
  FusedMlpArgs& a = b.a;
  a.X = X.data_ptr<float>();
  a.Yf = ptr_or_null<const float>(Yf);
  a.Yi = ptr_or_null<const int64_t>(Yi);
  a.P = P.data_ptr<float>();
  a.G = G.data_ptr<float>();
  a.mom = ptr_or_null<float>(mom);
  a.opt_step = ptr_or_null<int32_t>(opt_step);
  a.B = (int)B; a.Din = (int)Din; a.H = (int)H; a.Dout = (int)Dout;
  a.ldx = (int)X.stride(0);
  a.x_padded = x_zero_padded ? 1 : 0;
  a.loss_kind = (int)loss_kind;
  a.ignore_index = (int)ignore_index;
  a.has_bias = has_bias ? 1 : 0;
  a.grad_scale = 1.f;
  a.update_mode = 2;
  a.lr = (float)lr; a.momentum = (float)momentum; a.dampening = (float)dampening;
  a.weight_decay = (float)weight_decay; a.nesterov = nesterov ? 1 : 0;
  if (ar && ar->world() > 1) {
    TORCH_CHECK(ar->ready(), "persistent: xGMI communicator not opened");
    TORCH_CHECK(np <= ar->max_elems(), "persistent: bucket larger than the xGMI buffer");
    TORCH_CHECK(ar->rank() == rank, "persistent: rank mismatch");
    a.ar = ar->args();
  } else {
    a.ar.world = 1;
  }
  PersistArgs& pa = b.pa;
  pa.n_steps = (int)n_steps;
  pa.N = (int)N;
  pa.W = (int)W;
  pa.rank = (int)rank;
  pa.num_samples = (int)num_samples;
  pa.shuffle = shuffle ? 1 : 0;
  pa.seed = (uint64_t)seed;
  pa.cursor = cursor.data_ptr<int32_t>();
  pa.losses = losses.data_ptr<float>();
  if (stamps.has_value() && stamps->defined()) {
    TORCH_CHECK(stamps->is_cuda() && stamps->scalar_type() == at::kLong && stamps->numel() >= 9, "stamps: int64[9]");
    pa.stamps = stamps->data_ptr<int64_t>();
    pa.stamps_n = (int)stamps->numel();
  }
  pa.variant = (int)variant;
  pa.cursor_host_pos = -1;
  if (idx.has_value() && idx->defined()) {
    // [num_samples] (one epoch: cursor_j is the step in it) or [E, num_samples]
    // (epochs idx_e0..idx_e0+E-1: cursor_j is the absolute position epoch * S + step)
    TORCH_CHECK(idx->is_cuda() && idx->scalar_type() == at::kInt && idx->is_contiguous() &&
                    idx->size(-1) == num_samples && idx->dim() <= 2 && idx->device() == X.device(),
                "persistent: idx must be a contiguous int32 GPU tensor [E,] num_samples on X's device");
    const int64_t S = (num_samples + B - 1) / B;
    pa.idx = idx->data_ptr<int32_t>();
    pa.idx_epochs = idx->dim() == 2 ? (int)idx->size(0) : 1;
    pa.idx_e0 = idx->dim() == 2 ? (int)idx_e0 : 0;
    TORCH_CHECK(cursor_j >= (int64_t)pa.idx_e0 * S && cursor_j + n_steps <= (int64_t)(pa.idx_e0 + pa.idx_epochs) * S,
                "persistent: with explicit index lists a launch must stay inside the provided epochs");
    pa.cursor_host_pos = cursor_j;
  }
  if (lcache.has_value() && lcache->defined()) {  // [2][al4(num_samples)] lists + [2] epoch tags
    const int64_t stride = (num_samples + 3) & ~int64_t(3);
    TORCH_CHECK(lcache->is_cuda() && lcache->scalar_type() == at::kInt && lcache->is_contiguous() &&
                    lcache->numel() == 2 * stride + 2 && lcache->device() == X.device(),
                "persistent: list cache must be int32[2 * al4(num_samples) + 2] on X's device");
    pa.lcache = lcache->data_ptr<int32_t>();
    pa.ltag = pa.lcache + 2 * stride;
  }
  const bool wave = variant != kPersistWorkgroup && variant != kPersistMfma && variant != kPersistTp &&
                    variant != kPersistTpBf16 && linear_wave_supported(a, pa);
  const bool tp = !wave && (variant == kPersistAuto || variant == kPersistTp || variant == kPersistTpBf16) && H > 0 &&
                  mlp_tp_supported(a, pa);
  const bool mfma = !wave && !tp && mlp_mfma_persistent_supported(a, pa);
  TORCH_CHECK(wave || mfma || tp || (variant < kPersistWave),
              "persistent: the requested engine variant does not support this configuration");
  TORCH_CHECK(wave || tp || fused_mlp_persistent_lds_bytes((int)B, (int)Din, (int)H, (int)Dout, (int)num_samples,
                                                           world) <= 160 * 1024,
              "persistent: model + epoch index list do not fit one workgroup's LDS");
  return b;
}

void fused_mlp_persistent_py(Tensor X, c10::optional<Tensor> Yf, c10::optional<Tensor> Yi, Tensor P, Tensor G,
                             c10::optional<Tensor> mom, c10::optional<Tensor> opt_step, int64_t B, int64_t Din,
                             int64_t H, int64_t Dout, int64_t loss_kind, int64_t ignore_index, bool has_bias,
                             double lr, double momentum, double dampening, double weight_decay, bool nesterov,
                             std::shared_ptr<XgmiComm> ar, int64_t n_steps, int64_t W, int64_t rank,
                             int64_t num_samples, bool shuffle, int64_t seed, Tensor cursor, Tensor losses,
                             c10::optional<Tensor> stamps, int64_t variant, bool x_zero_padded,
                             c10::optional<Tensor> idx, int64_t cursor_j) {
  const PersistBuild b = build_persistent(X, Yf, Yi, P, G, mom, opt_step, B, Din, H, Dout, loss_kind, ignore_index,
                                          has_bias, lr, momentum, dampening, weight_decay, nesterov, ar, n_steps, W,
                                          rank, num_samples, shuffle, seed, cursor, losses, stamps, variant,
                                          x_zero_padded, idx, cursor_j);
  c10::hip::HIPGuard guard(X.device().index());
  hip_check(fused_mlp_persistent(b.a, b.pa, cur_stream(X)), "fused_mlp_persistent");
}

// A persistent engine launch planned once: arguments validated, engine and
// kernel chosen, LDS attribute set, tensors kept alive. launch(n) is a bare
// hipLaunchKernel on the caller's current stream -- the short-run fixed cost
// (bench --steps 20, one launch per Trainer.train) is the kernel, not the host.
int64_t mono_ns() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (int64_t)t.tv_sec * 1000000000 + t.tv_nsec;
}

class PersistentPlan {
 public:
  PersistentPlan(Tensor X, c10::optional<Tensor> Yf, c10::optional<Tensor> Yi, Tensor P, Tensor G,
                 c10::optional<Tensor> mom, c10::optional<Tensor> opt_step, int64_t B, int64_t Din, int64_t H,
                 int64_t Dout, int64_t loss_kind, int64_t ignore_index, bool has_bias, double lr, double momentum,
                 double dampening, double weight_decay, bool nesterov, std::shared_ptr<XgmiComm> ar, int64_t W,
                 int64_t rank, int64_t num_samples, bool shuffle, int64_t seed, Tensor cursor, Tensor losses,
                 c10::optional<Tensor> stamps, int64_t variant, bool x_zero_padded, c10::optional<Tensor> idx,
                 c10::optional<Tensor> lcache, int64_t idx_e0)
      : keep_{X, P, G, cursor, losses}, ar_(ar), capacity_(losses.numel()), dev_(X.device().index()) {
    for (const auto* t : {&Yf, &Yi, &mom, &opt_step, &stamps, &idx, &lcache})
      if (t->has_value() && (*t)->defined()) keep_.push_back(**t);
    const bool has_idx = idx.has_value() && idx->defined();
    steps_per_epoch_ = (num_samples + B - 1) / B;
    const int64_t first = has_idx && idx->dim() == 2 ? idx_e0 * steps_per_epoch_ : 0;
    const PersistBuild b = build_persistent(X, Yf, Yi, P, G, mom, opt_step, B, Din, H, Dout, loss_kind, ignore_index,
                                            has_bias, lr, momentum, dampening, weight_decay, nesterov, ar, 1, W, rank,
                                            num_samples, shuffle, seed, cursor, losses, stamps, variant,
                                            x_zero_padded, idx, has_idx ? first : -1, lcache, idx_e0);
    c10::hip::HIPGuard guard(dev_);
    hip_check(fused_mlp_persistent_prepare(b.a, b.pa, &L_), "persistent plan");
  }
  // n steps from the device cursor; with explicit index lists, cursor_pos is
  // the host's view of the cursor (epoch * steps_per_epoch + step; one-epoch
  // list: the step in it) and the launch must stay inside the provided epochs
  void launch(int64_t n, int64_t cursor_pos) { launch_impl(n, cursor_pos, -1, 0); }
  void launch_impl(int64_t n, int64_t cursor_pos, int start_e, int start_j) {
    TORCH_CHECK(n >= 0 && n <= capacity_, "persistent plan: n_steps exceeds the losses buffer");
    const int64_t S = steps_per_epoch_;
    TORCH_CHECK(L_.p.idx == nullptr || (cursor_pos >= (int64_t)L_.p.idx_e0 * S &&
                                        cursor_pos + n <= (int64_t)(L_.p.idx_e0 + L_.p.idx_epochs) * S),
                "persistent plan: with explicit index lists a launch must stay inside the provided epochs");
    c10::hip::HIPGuard guard(dev_);
    hip_check(persistent_launch(L_, (int)n, L_.p.idx ? cursor_pos : -1, c10::hip::getCurrentHIPStream(dev_).stream(),
                                start_e, start_j),
              "persistent launch");
  }
  // n steps from absolute position pos = epoch * steps_per_epoch + step, which the
  // caller asserts the device cursor holds (its own step count, e.g. the bench's
  // warm-up): the engines skip the dependent cursor load at kernel entry
  void launch_at(int64_t n, int64_t pos) {
    TORCH_CHECK(pos >= 0, "persistent plan: launch_at needs a position >= 0");
    const int64_t S = steps_per_epoch_;
    TORCH_CHECK(pos / S < (int64_t)1 << 30, "persistent plan: position out of range");
    launch_impl(n, pos, (int)(pos / S), (int)(pos % S));
  }
  int64_t capacity() const { return capacity_; }
  ~PersistentPlan() {
    if (ev_) hipEventDestroy(ev_);
  }
  // launch timeline probe (tools/driver_timeline.py): the engine stamps its realtime counter
  // into tl[0..3] (a device or host-mapped int64 address; 0 turns it off)
  void set_timeline(int64_t addr) { L_.p.tl = reinterpret_cast<int64_t*>(addr); }
  // CLOCK_MONOTONIC ns right before / after the last hipLaunchKernel of this plan
  std::vector<int64_t> last_launch_ns() const { return {L_.host_ns[0], L_.host_ns[1]}; }
  // Timeline probe: launch n steps at pos and wait for them with one of the runtime's completion
  // paths, all in C++ (mode 0 hipDeviceSynchronize, 1 hipStreamSynchronize, 2 hipEventRecord +
  // hipEventSynchronize, 3 hipExtLaunchKernel with a stop event + hipEventSynchronize, 4 spin on
  // hipStreamQuery, 5 hipExtLaunchKernel with a stop event + spin on hipEventQuery). Returns
  // CLOCK_MONOTONIC ns [before the launch call, after it, when the wait returned].
  std::vector<int64_t> launch_wait_at(int64_t n, int64_t pos, int64_t mode) {
    TORCH_CHECK(n > 0 && n <= capacity_ && pos >= 0, "launch_wait_at: bad n / pos");
    TORCH_CHECK(mode >= 0 && mode <= 5, "launch_wait_at: mode 0..5");
    const int64_t S = steps_per_epoch_;
    c10::hip::HIPGuard guard(dev_);
    hipStream_t st = c10::hip::getCurrentHIPStream(dev_).stream();
    if (ev_ == nullptr) hip_check(hipEventCreate(&ev_), "hipEventCreate");
    const int64_t t0 = mono_ns();
    if (mode == 3 || mode == 5) {
      L_.p.n_steps = (int)n;
      L_.p.cursor_host_pos = -1;
      L_.p.has_start = 1;
      L_.p.start_e = (int)(pos / S);
      L_.p.start_j = (int)(pos % S);
      void* args[] = {&L_.a, &L_.p};
      hip_check(hipExtLaunchKernel(L_.fn, dim3(1), dim3(L_.threads), args, L_.lds, st, nullptr, ev_, 0),
                "hipExtLaunchKernel");
    } else {
      launch_impl(n, pos, (int)(pos / S), (int)(pos % S));
      if (mode == 2) hip_check(hipEventRecord(ev_, st), "hipEventRecord");
    }
    const int64_t t1 = mono_ns();
    switch (mode) {
      case 0: hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize"); break;
      case 1: hip_check(hipStreamSynchronize(st), "hipStreamSynchronize"); break;
      case 2:
      case 3: hip_check(hipEventSynchronize(ev_), "hipEventSynchronize"); break;
      case 4: {
        hipError_t e;
        while ((e = hipStreamQuery(st)) == hipErrorNotReady) {
        }
        hip_check(e, "hipStreamQuery");
        break;
      }
      default: {
        hipError_t e;
        while ((e = hipEventQuery(ev_)) == hipErrorNotReady) {
        }
        hip_check(e, "hipEventQuery");
      }
    }
    return {t0, t1, mono_ns()};
  }

 private:
  std::vector<Tensor> keep_;
  std::shared_ptr<XgmiComm> ar_;
  int64_t capacity_;
  int dev_;
  int64_t steps_per_epoch_ = 0;
  PersistLaunch L_;
  hipEvent_t ev_ = nullptr;  // timeline probe (launch_wait_at)
};

// Host-mapped, coherent int64 words a kernel can store into and the host can poll
// (launch timelines: tools/driver_timeline.py).
class HostMapped {
 public:
  explicit HostMapped(int64_t n) : n_(n) {
    TORCH_CHECK(n > 0 && n <= (1 << 20), "HostMapped: 1..2^20 words");
    hip_check(hipHostMalloc((void**)&h_, n * sizeof(int64_t), hipHostMallocMapped | hipHostMallocCoherent),
              "hipHostMalloc(HostMapped)");
    hip_check(hipHostGetDevicePointer((void**)&d_, h_, 0), "hipHostGetDevicePointer(HostMapped)");
    zero();
  }
  ~HostMapped() {
    if (h_) hipHostFree(h_);
  }
  HostMapped(const HostMapped&) = delete;
  HostMapped& operator=(const HostMapped&) = delete;
  void zero() {
    volatile int64_t* v = h_;
    for (int64_t k = 0; k < n_; ++k) v[k] = 0;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
  }
  std::vector<int64_t> read() const {
    volatile int64_t* v = h_;
    std::vector<int64_t> out(n_);
    for (int64_t k = 0; k < n_; ++k) out[k] = v[k];
    return out;
  }
  // spin until word k is non-zero; CLOCK_MONOTONIC ns when it was seen, -1 after timeout_ns
  int64_t spin(int64_t k, int64_t timeout_ns) const {
    TORCH_CHECK(k >= 0 && k < n_);
    volatile int64_t* v = h_ + k;
    const int64_t t0 = mono_ns();
    for (;;) {
      if (*v != 0) return mono_ns();
      const int64_t t = mono_ns();
      if (t - t0 > timeout_ns) return -1;
    }
  }
  int64_t device_ptr() const { return reinterpret_cast<int64_t>(d_); }

 private:
  int64_t n_;
  int64_t* h_ = nullptr;
  int64_t* d_ = nullptr;
};

std::vector<std::vector<int64_t>> clock_calibrate_py(int64_t n) {
  std::vector<int64_t> a(n), b(n), c(n);
  hip_check(clock_calibrate((int)n, a.data(), b.data(), c.data()), "clock_calibrate");
  return {a, b, c};
}

// Which persistent engine fused_mlp_persistent would run for this configuration
// ("workgroup", or "wave:L<lanes per row>R<rows per lane group>K<features per lane>").
std::string persistent_engine(int64_t B, int64_t Din, int64_t H, int64_t Dout, int64_t loss_kind, int64_t num_samples,
                              int64_t world, int64_t variant, bool has_bias) {
  FusedMlpArgs a{};
  a.B = (int)B; a.Din = (int)Din; a.H = (int)H; a.Dout = (int)Dout; a.loss_kind = (int)loss_kind;
  a.has_bias = has_bias ? 1 : 0;
  a.ar.world = (int)world;
  a.ldx = kWaveLdxAny;  // the caller zero-pads X rows to the layout's width when needed
  a.x_padded = 1;
  PersistArgs pa{};
  pa.num_samples = (int)num_samples;
  pa.variant = (int)variant;
  pa.N = (int)std::max<int64_t>(num_samples, 1);
  if (variant != kPersistWorkgroup && variant != kPersistMfma && variant != kPersistTp && variant != kPersistTpBf16 &&
      linear_wave_supported(a, pa)) {
    int L = 0, R = 0, kp = 0;
    linear_wave_layout(a, pa, &L, &R, &kp);
    return "wave:L" + std::to_string(L) + "R" + std::to_string(R) + "K" + std::to_string(kp);
  }
  if (variant == kPersistTpBf16 && H > 0 && mlp_tp_supported(a, pa)) return "tp_bf16:" + std::to_string(H / 16) + "waves";
  if ((variant == kPersistAuto || variant == kPersistTp) && H > 0 && mlp_tp_supported(a, pa))
    return "tp:" + std::to_string(H / 16) + "waves";
  if (variant != kPersistWorkgroup && mlp_mfma_persistent_supported(a, pa)) return "workgroup:mfma";
  return "workgroup";
}

// ------------------------------------------------------------- torch-identical sampler orders
void torch_perm_py(Tensor seeds, int64_t n, int64_t W, int64_t rank, int64_t num_samples, Tensor out,
                   c10::optional<Tensor> ws) {
  check_gpu(seeds, "seeds");
  check_gpu(out, "out");
  TORCH_CHECK(seeds.scalar_type() == at::kLong && seeds.dim() == 1, "torch_perm: seeds int64[E]");
  TORCH_CHECK(out.scalar_type() == at::kInt && out.dim() == 2 && out.size(0) == seeds.size(0) &&
                  out.size(1) >= num_samples && out.device() == seeds.device(),
              "torch_perm: out int32[E, >= num_samples] on the seeds' device");
  TORCH_CHECK(n >= 2 && n < (1ll << 31) && W > 0 && rank >= 0 && rank < W && num_samples > 0,
              "torch_perm: bad sampler geometry");
  int32_t* wsp = nullptr;
  if (torch_perm_lds_bytes((int)n) + 624 * 4 > 160 * 1024) {
    TORCH_CHECK(ws.has_value() && ws->defined() && ws->is_cuda() && ws->scalar_type() == at::kInt &&
                    ws->is_contiguous() && ws->numel() >= seeds.size(0) * 4 * n,
                "torch_perm: n too large for LDS, pass ws = int32[E * 4n]");
    wsp = ws->data_ptr<int32_t>();
  }
  c10::hip::HIPGuard guard(out.device().index());
  hip_check(torch_perm(seeds.data_ptr<int64_t>(), (int)seeds.size(0), (int)n, (int)W, (int)rank, (int)num_samples,
                       out.data_ptr<int32_t>(), (int)out.size(1), wsp, cur_stream(out)),
            "torch_perm");
}

// ------------------------------------------------------------- optimizers
void sgd_flat_(Tensor p, Tensor g, c10::optional<Tensor> mom, c10::optional<Tensor> step, double lr,
               double momentum, double dampening, double wd, bool nesterov, double grad_scale) {
  check_gpu(p, "param");
  check_gpu(g, "grad");
  TORCH_CHECK(p.scalar_type() == at::kFloat && g.scalar_type() == at::kFloat && p.numel() == g.numel());
  c10::hip::HIPGuard guard(p.device().index());
  hip_check(sgd_flat(p.data_ptr<float>(), g.data_ptr<float>(), ptr_or_null<float>(mom),
                     ptr_or_null<int32_t>(step), p.numel(), (float)lr, (float)momentum, (float)dampening,
                     (float)wd, nesterov, (float)grad_scale, cur_stream(p)),
            "sgd_flat");
}

void adam_flat_(Tensor p, Tensor g, Tensor m, Tensor v, Tensor step, double lr, double b1, double b2,
                double eps, double wd, bool decoupled, double grad_scale) {
  check_gpu(p, "param");
  TORCH_CHECK(p.scalar_type() == at::kFloat && g.numel() == p.numel() && m.numel() == p.numel() &&
              v.numel() == p.numel() && step.scalar_type() == at::kInt);
  c10::hip::HIPGuard guard(p.device().index());
  hip_check(adam_flat(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                      step.data_ptr<int32_t>(), p.numel(), (float)lr, (float)b1, (float)b2, (float)eps,
                      (float)wd, decoupled, (float)grad_scale, cur_stream(p)),
            "adam_flat");
}

template <typename F>
void for_tensor_chunks(size_t n, F&& f) {
  for (size_t s = 0; s < n; s += kMaxTensorsPerLaunch) f(s, std::min(n, s + (size_t)kMaxTensorsPerLaunch));
}

void sgd_multi_(std::vector<Tensor> ps, std::vector<Tensor> gs, std::vector<Tensor> moms,
                c10::optional<Tensor> step, double lr, double momentum, double dampening, double wd,
                bool nesterov, double grad_scale, std::vector<Tensor> shadows) {
  if (ps.empty()) return;
  TORCH_CHECK(ps.size() == gs.size() && (moms.empty() || moms.size() == ps.size()));
  TORCH_CHECK(shadows.empty() || (shadows.size() == ps.size() && ps[0].scalar_type() == at::kFloat),
              "sgd_multi_: bf16 shadows need one per (f32) param");
  const int dt = dt_of(ps[0]);
  c10::hip::HIPGuard guard(ps[0].device().index());
  for_tensor_chunks(ps.size(), [&](size_t a, size_t b) {
    TensorList tl{};
    tl.n = (int)(b - a);
    for (size_t i = a; i < b; ++i) {
      check_dense_like(ps[i], ps[i], "param");
      check_dense_like(ps[i], gs[i], "grad");
      if (!moms.empty()) check_dense_like(ps[i], moms[i], "momentum buffer");
      TORCH_CHECK(dt_of(ps[i]) == dt && gs[i].scalar_type() == ps[i].scalar_type() && gs[i].numel() == ps[i].numel());
      tl.numel[i - a] = ps[i].numel();
      tl.p[i - a] = ps[i].data_ptr();
      tl.g[i - a] = gs[i].data_ptr();
      tl.s1[i - a] = moms.empty() ? nullptr : moms[i].data_ptr<float>();
      tl.s2[i - a] = nullptr;
      if (!shadows.empty()) {
        TORCH_CHECK(shadows[i].scalar_type() == at::kBFloat16 && shadows[i].numel() == ps[i].numel(),
                    "sgd_multi_: shadow must be a bf16 tensor of the param's size");
        check_dense_like(ps[i], shadows[i], "bf16 shadow");
        tl.s2[i - a] = reinterpret_cast<float*>(shadows[i].data_ptr());
      }
    }
    hip_check(sgd_multi(tl, dt, ptr_or_null<int32_t>(step), (float)lr, (float)momentum, (float)dampening,
                        (float)wd, nesterov, (float)grad_scale, cur_stream(ps[0])),
              "sgd_multi");
  });
}

void adam_multi_(std::vector<Tensor> ps, std::vector<Tensor> gs, std::vector<Tensor> ms,
                 std::vector<Tensor> vs, Tensor step, double lr, double b1, double b2, double eps,
                 double wd, bool decoupled, double grad_scale) {
  if (ps.empty()) return;
  TORCH_CHECK(ps.size() == gs.size() && ms.size() == ps.size() && vs.size() == ps.size());
  const int dt = dt_of(ps[0]);
  c10::hip::HIPGuard guard(ps[0].device().index());
  for_tensor_chunks(ps.size(), [&](size_t a, size_t b) {
    TensorList tl{};
    tl.n = (int)(b - a);
    for (size_t i = a; i < b; ++i) {
      check_dense_like(ps[i], ps[i], "param");
      check_dense_like(ps[i], gs[i], "grad");
      check_dense_like(ps[i], ms[i], "exp_avg");
      check_dense_like(ps[i], vs[i], "exp_avg_sq");
      TORCH_CHECK(dt_of(ps[i]) == dt && gs[i].numel() == ps[i].numel());
      TORCH_CHECK(ms[i].scalar_type() == at::kFloat && vs[i].scalar_type() == at::kFloat);
      tl.numel[i - a] = ps[i].numel();
      tl.p[i - a] = ps[i].data_ptr();
      tl.g[i - a] = gs[i].data_ptr();
      tl.s1[i - a] = ms[i].data_ptr<float>();
      tl.s2[i - a] = vs[i].data_ptr<float>();
    }
    hip_check(adam_multi(tl, dt, step.data_ptr<int32_t>(), (float)lr, (float)b1, (float)b2, (float)eps,
                         (float)wd, decoupled, (float)grad_scale, cur_stream(ps[0])),
              "adam_multi");
  });
}

void bucket_copy(std::vector<Tensor> ts, Tensor flat, double scale, bool unpack) {
  if (ts.empty()) return;
  check_gpu(flat, "flat");
  const int dt = dt_of(flat);
  c10::hip::HIPGuard guard(flat.device().index());
  int64_t off = 0;
  for_tensor_chunks(ts.size(), [&](size_t a, size_t b) {
    CopyList cl{};
    cl.n = (int)(b - a);
    for (size_t i = a; i < b; ++i) {
      check_gpu(ts[i], "tensor");
      TORCH_CHECK(ts[i].scalar_type() == flat.scalar_type());
      cl.numel[i - a] = ts[i].numel();
      cl.offset[i - a] = off;
      cl.t[i - a] = ts[i].data_ptr();
      off += ts[i].numel();
    }
    TORCH_CHECK(off <= flat.numel(), "bucket_copy: flat buffer too small");
    hip_check(unpack ? bucket_unpack(cl, flat.data_ptr(), dt, (float)scale, cur_stream(flat))
                     : bucket_pack(cl, flat.data_ptr(), dt, (float)scale, cur_stream(flat)),
              "bucket_copy");
  });
}

// dsts[i] (f32) = srcs[i] (bf16), one multi-tensor launch per <= 32 pairs; pairs must share shape and strides
void cast_multi_(std::vector<Tensor> dsts, std::vector<Tensor> srcs) {
  TORCH_CHECK(dsts.size() == srcs.size(), "cast_multi_: one source per destination");
  if (dsts.empty()) return;
  c10::hip::HIPGuard guard(dsts[0].device().index());
  for_tensor_chunks(dsts.size(), [&](size_t a, size_t b) {
    TensorList tl{};
    tl.n = (int)(b - a);
    for (size_t i = a; i < b; ++i) {
      TORCH_CHECK(dsts[i].scalar_type() == at::kFloat && srcs[i].scalar_type() == at::kBFloat16,
                  "cast_multi_: f32 destinations, bf16 sources");
      TORCH_CHECK(dsts[i].device() == dsts[0].device() && srcs[i].device() == dsts[0].device(),
                  "cast_multi_: one device");
      check_dense_like(dsts[i], dsts[i], "destination");
      check_dense_like(dsts[i], srcs[i], "source");
      tl.numel[i - a] = dsts[i].numel();
      tl.p[i - a] = dsts[i].data_ptr();
      tl.g[i - a] = srcs[i].data_ptr();
    }
    hip_check(cast_bf16_f32_multi(tl, cur_stream(dsts[0])), "cast_bf16_f32_multi");
  });
}

// [N, 3, H, W] channels_last f32/bf16 -> [N, 4, H, W] channels_last bf16 with a zero 4th channel
Tensor rgb4_pack_(Tensor x) {
  TORCH_CHECK(x.is_cuda(), "rgb4_pack: x must be a GPU tensor");
  TORCH_CHECK(x.dim() == 4 && x.size(1) == 3 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "rgb4_pack: x must be a channels_last [N, 3, H, W] tensor");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "rgb4_pack: f32 or bf16");
  c10::hip::HIPGuard guard(x.device().index());
  Tensor y = at::empty({x.size(0), 4, x.size(2), x.size(3)},
                       x.options().dtype(at::kBFloat16).memory_format(at::MemoryFormat::ChannelsLast));
  hip_check(rgb4_pack(x.data_ptr(), dt_of(x), static_cast<uint16_t*>(y.data_ptr()), x.numel() / 3, cur_stream(x)),
            "rgb4_pack");
  return y;
}

void scale_(Tensor x, double s) {
  check_gpu(x, "x");
  c10::hip::HIPGuard guard(x.device().index());
  hip_check(scale_inplace(x.data_ptr(), x.numel(), dt_of(x), (float)s, cur_stream(x)), "scale_inplace");
}

// ------------------------------------------------------------- losses
// returns (loss[1], lse_ws[3B], valid[1])
std::vector<Tensor> ce_fwd(Tensor logits, c10::optional<Tensor> soft, c10::optional<Tensor> index,
                           int64_t ignore_index, double label_smoothing) {
  check_gpu(logits, "logits");
  TORCH_CHECK(logits.dim() == 2, "cross_entropy: logits must be [B, C]");
  const int64_t B = logits.size(0), C = logits.size(1);
  if (soft.has_value() && soft->defined()) {
    check_gpu(*soft, "soft target");
    TORCH_CHECK(soft->scalar_type() == at::kFloat && soft->numel() == B * C, "soft targets: float [B, C]");
  } else {
    TORCH_CHECK(index.has_value() && index->defined(), "cross_entropy: need soft or index targets");
    check_gpu(*index, "index target");
    TORCH_CHECK(index->scalar_type() == at::kLong && index->numel() == B, "index targets: int64 [B]");
  }
  c10::hip::HIPGuard guard(logits.device().index());
  auto fopt = logits.options().dtype(at::kFloat);
  Tensor loss = at::empty({}, fopt), lse = at::empty({3 * B}, fopt), valid = at::empty({1}, fopt);
  hip_check(ce_forward(logits.data_ptr(), dt_of(logits), ptr_or_null<const float>(soft),
                       ptr_or_null<const int64_t>(index), (int)B, (int)C, (int)ignore_index,
                       (float)label_smoothing, loss.data_ptr<float>(), lse.data_ptr<float>(),
                       valid.data_ptr<float>(), cur_stream(logits)),
            "ce_forward");
  return {loss, lse, valid};
}

Tensor ce_bwd(Tensor logits, c10::optional<Tensor> soft, c10::optional<Tensor> index, Tensor lse,
              Tensor valid, c10::optional<Tensor> grad_out, int64_t ignore_index, double label_smoothing) {
  check_gpu(logits, "logits");
  const int64_t B = logits.size(0), C = logits.size(1);
  c10::hip::HIPGuard guard(logits.device().index());
  Tensor d = at::empty_like(logits);
  hip_check(ce_backward(logits.data_ptr(), dt_of(logits), ptr_or_null<const float>(soft),
                        ptr_or_null<const int64_t>(index), lse.data_ptr<float>(), valid.data_ptr<float>(),
                        ptr_or_null<const float>(grad_out), (int)B, (int)C, (int)ignore_index,
                        (float)label_smoothing, d.data_ptr(), cur_stream(logits)),
            "ce_backward");
  return d;
}

Tensor mse_fwd(Tensor x, Tensor y) {
  check_gpu(x, "input");
  check_gpu(y, "target");
  TORCH_CHECK(x.numel() == y.numel() && x.scalar_type() == y.scalar_type(), "mse: shape/dtype mismatch");
  c10::hip::HIPGuard guard(x.device().index());
  Tensor ws = at::empty({1 + 1024}, x.options().dtype(at::kFloat));
  hip_check(mse_forward(x.data_ptr(), y.data_ptr(), dt_of(x), x.numel(), ws.data_ptr<float>(), cur_stream(x)),
            "mse_forward");
  return ws.narrow(0, 0, 1).reshape({}).clone();
}

std::vector<Tensor> mse_bwd(Tensor x, Tensor y, c10::optional<Tensor> grad_out, bool need_dx, bool need_dy) {
  check_gpu(x, "input");
  check_gpu(y, "target");
  c10::hip::HIPGuard guard(x.device().index());
  Tensor dx = need_dx ? at::empty_like(x) : Tensor();
  Tensor dy = need_dy ? at::empty_like(y) : Tensor();
  hip_check(mse_backward(x.data_ptr(), y.data_ptr(), dt_of(x), x.numel(), ptr_or_null<const float>(grad_out),
                         need_dx ? dx.data_ptr() : nullptr, need_dy ? dy.data_ptr() : nullptr, cur_stream(x)),
            "mse_backward");
  return {dx, dy};
}

// ------------------------------------------------------------- GEMM / Linear
// C = alpha*A.B (+beta C) (+bias) (relu); A/B/C/mask are 2-D (possibly transposed views).
void gemm_(Tensor A, Tensor B, Tensor C, c10::optional<Tensor> bias, c10::optional<Tensor> amask, bool relu,
           double alpha, double beta, c10::optional<Tensor> colsum, int64_t split_k) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && C.is_cuda(), "gemm: GPU tensors");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && C.dim() == 2, "gemm: 2-D operands");
  TORCH_CHECK(A.size(1) == B.size(0) && C.size(0) == A.size(0) && C.size(1) == B.size(1), "gemm: shape mismatch ",
              A.sizes(), " x ", B.sizes(), " -> ", C.sizes());
  TORCH_CHECK(A.scalar_type() == B.scalar_type(), "gemm: A/B dtype mismatch");
  GemmArgs g{};
  g.M = (int)A.size(0);
  g.N = (int)B.size(1);
  g.K = (int)A.size(1);
  g.A = A.data_ptr(); g.sam = A.stride(0); g.sak = A.stride(1);
  g.B = B.data_ptr(); g.sbk = B.stride(0); g.sbn = B.stride(1);
  g.C = C.data_ptr(); g.scm = C.stride(0); g.scn = C.stride(1);
  g.in_dtype = dt_of(A);
  g.out_dtype = dt_of(C);
  if (bias.has_value() && bias->defined()) {
    check_gpu(*bias, "bias");
    TORCH_CHECK(bias->numel() == g.N, "gemm: bias must have N entries");
    g.bias = bias->data_ptr();
    g.bias_dtype = dt_of(*bias);
  }
  if (amask.has_value() && amask->defined()) {
    TORCH_CHECK(amask->sizes() == A.sizes() && amask->scalar_type() == A.scalar_type(), "gemm: mask like A");
    g.amask = amask->data_ptr(); g.smm = amask->stride(0); g.smk = amask->stride(1);
  }
  if (colsum.has_value() && colsum->defined()) {
    check_gpu(*colsum, "colsum");
    TORCH_CHECK(colsum->scalar_type() == at::kFloat && colsum->numel() == g.M, "gemm: colsum f32 [M]");
    g.colsum_out = colsum->data_ptr<float>();
  }
  g.relu = relu ? 1 : 0;
  g.alpha = (float)alpha;
  g.beta = (float)beta;
  g.split_k = (int)split_k;
  c10::hip::HIPGuard guard(A.device().index());
  hip_check(gemm(g, cur_stream(A)), "gemm");
}

// C = alpha*A.Bt^T (+beta C) (+bias) (relu) on the LDS-DMA kernel (gemm_big.hip): 256x256 or 128x128
// block tile, optional split-K (f32 C pre-zeroed by the caller).
// A [M,K], Bt [N,K]: bf16 with unit K stride; C [M,N] f32/bf16 with unit column stride.
bool gemm_big_ok(Tensor A, Tensor Bt) {
  return A.is_cuda() && Bt.is_cuda() && A.dim() == 2 && Bt.dim() == 2 && A.scalar_type() == at::kBFloat16 &&
         Bt.scalar_type() == at::kBFloat16 && A.stride(1) == 1 && Bt.stride(1) == 1 && A.size(1) == Bt.size(1) &&
         gemm_bf16_big_supported((int)A.size(0), (int)Bt.size(0), (int)A.size(1), A.stride(0), Bt.stride(0),
                                 A.data_ptr(), Bt.data_ptr());
}

void gemm_big_(Tensor A, Tensor Bt, Tensor C, c10::optional<Tensor> bias, bool relu, double alpha, double beta,
               int64_t sched, int64_t tile, int64_t split_k) {
  TORCH_CHECK(gemm_big_ok(A, Bt), "gemm_big: needs bf16 A[M,K], Bt[N,K] with unit K stride, K % 64 == 0, "
              "16-B aligned rows; got ", A.sizes(), A.strides(), " / ", Bt.sizes(), Bt.strides());
  TORCH_CHECK(C.is_cuda() && C.dim() == 2 && C.size(0) == A.size(0) && C.size(1) == Bt.size(0) && C.stride(1) == 1,
              "gemm_big: C must be [M,N] with unit column stride");
  TORCH_CHECK(C.scalar_type() == at::kFloat || C.scalar_type() == at::kBFloat16, "gemm_big: C f32 or bf16");
  BigGemmArgs g{};
  g.M = (int)A.size(0);
  g.N = (int)Bt.size(0);
  g.K = (int)A.size(1);
  g.A = A.data_ptr(); g.lda = A.stride(0);
  g.Bt = Bt.data_ptr(); g.ldb = Bt.stride(0);
  g.C = C.data_ptr(); g.ldc = C.stride(0);
  g.out_dtype = dt_of(C);
  if (bias.has_value() && bias->defined()) {
    check_gpu(*bias, "bias");
    TORCH_CHECK(bias->numel() == g.N, "gemm_big: bias must have N entries");
    g.bias = bias->data_ptr();
    g.bias_dtype = dt_of(*bias);
  }
  g.relu = relu ? 1 : 0;
  g.alpha = (float)alpha;
  g.beta = (float)beta;
  g.tile = tile == 128 ? 128 : 256;
  g.sched = sched < 0 ? (g.tile == 256 ? 4 : 0) : (int)sched;  // 256 tile: 8-phase schedule, grouped tile order
  g.split_k = split_k > 1 ? (int)split_k : 1;
  TORCH_CHECK(g.split_k == 1 || (C.scalar_type() == at::kFloat && !relu && beta == 0.0),
              "gemm_big: split-K accumulates fp32 atomics: C must be f32 (pre-zeroed), no relu/beta");
  c10::hip::HIPGuard guard(A.device().index());
  hip_check(gemm_bf16_big(g, cur_stream(A)), "gemm_big");
}

Tensor relu_bwd(Tensor dy, Tensor y) {
  check_gpu(dy, "dy");
  check_gpu(y, "y");
  c10::hip::HIPGuard guard(dy.device().index());
  Tensor dx = at::empty_like(dy);
  hip_check(relu_backward(dy.data_ptr(), y.data_ptr(), dx.data_ptr(), dt_of(dy), dy.numel(), cur_stream(dy)),
            "relu_backward");
  return dx;
}

Tensor sum_all_(Tensor x) {
  check_gpu(x, "x");
  auto out = torch::empty({}, x.options().dtype(at::kFloat));
  c10::hip::HIPGuard guard(x.device().index());
  hip_check(sum_all(x.data_ptr(), dt_of(x), x.numel(), out.data_ptr<float>(), cur_stream(x)), "sum_all");
  return out;
}

void col_sum_(Tensor x, Tensor out, bool accumulate) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 2 && out.scalar_type() == at::kFloat && out.numel() == x.size(1));
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.device() == x.device(), "col_sum_: out must be on x's device");
  c10::hip::HIPGuard guard(x.device().index());
  const int nsplit = col_sum_splits(x.size(0), x.size(1));
  Tensor ws = nsplit > 1 ? at::empty({nsplit, x.size(1)}, out.options()) : Tensor();
  hip_check(col_sum(x.data_ptr(), dt_of(x), x.size(0), x.size(1), out.data_ptr<float>(), accumulate,
                    nsplit > 1 ? ws.data_ptr<float>() : nullptr, nsplit, cur_stream(x)),
            "col_sum");
}

// ------------------------------------------------------------- data
void philox_(Tensor out, int64_t seed, int64_t offset, int64_t dist) {
  check_gpu(out, "out");
  TORCH_CHECK(out.scalar_type() == at::kFloat);
  c10::hip::HIPGuard guard(out.device().index());
  hip_check(philox_fill(out.data_ptr<float>(), out.numel(), (uint64_t)seed, (uint64_t)offset, (int)dist,
                        cur_stream(out)),
            "philox_fill");
}

Tensor one_hot_(Tensor idx, int64_t C) {
  check_gpu(idx, "idx");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.dim() == 1);
  c10::hip::HIPGuard guard(idx.device().index());
  Tensor out = at::empty({idx.size(0), C}, idx.options().dtype(at::kFloat));
  hip_check(one_hot(idx.data_ptr<int64_t>(), out.data_ptr<float>(), (int)idx.size(0), (int)C, cur_stream(idx)),
            "one_hot");
  return out;
}

void gather_rows_(Tensor src, Tensor idx, Tensor out) {
  check_gpu(src, "src");
  check_gpu(idx, "idx");
  check_gpu(out, "out");
  TORCH_CHECK(idx.scalar_type() == at::kInt && out.scalar_type() == src.scalar_type());
  TORCH_CHECK(src.dim() >= 1 && out.size(0) == idx.numel(), "gather_rows: out rows == idx count");
  const int64_t cols = src.numel() / std::max<int64_t>(src.size(0), 1);
  TORCH_CHECK(out.numel() == idx.numel() * cols);
  c10::hip::HIPGuard guard(src.device().index());
  hip_check(gather_rows(src.data_ptr(), idx.data_ptr<int32_t>(), out.data_ptr(), idx.numel(), cols,
                        (int)src.element_size(), cur_stream(src)),
            "gather_rows");
}

void device_sampler_(Tensor out, int64_t N, int64_t W, int64_t rank, int64_t num_samples, int64_t seed,
                     Tensor epoch, bool shuffle) {
  check_gpu(out, "out");
  TORCH_CHECK(out.scalar_type() == at::kInt && out.numel() >= num_samples, "sampler out: int32 [num_samples]");
  TORCH_CHECK(epoch.is_cuda() && epoch.scalar_type() == at::kInt && epoch.numel() == 1, "epoch: int32 [1] on GPU");
  TORCH_CHECK(N > 0 && W > 0 && rank >= 0 && rank < W, "device_sampler: bad N/W/rank");
  c10::hip::HIPGuard guard(out.device().index());
  hip_check(device_sampler(out.data_ptr<int32_t>(), N, (int)W, (int)rank, num_samples, (uint64_t)seed,
                           epoch.data_ptr<int32_t>(), shuffle ? 1 : 0, cur_stream(out)),
            "device_sampler");
}

// ------------------------------------------------------------- int8
std::vector<Tensor> quantize_int8(Tensor w) {
  check_gpu(w, "weight");
  TORCH_CHECK(w.dim() == 2);
  c10::hip::HIPGuard guard(w.device().index());
  Tensor q = at::empty(w.sizes(), w.options().dtype(at::kChar));
  Tensor s = at::empty({w.size(0)}, w.options().dtype(at::kFloat));
  hip_check(quantize_rowwise_int8(w.data_ptr(), dt_of(w), w.size(0), w.size(1), q.data_ptr<int8_t>(),
                                  s.data_ptr<float>(), cur_stream(w)),
            "quantize_int8");
  return {q, s};
}

Tensor int8_linear(Tensor x, Tensor q, Tensor scale, c10::optional<Tensor> bias) {
  check_gpu(x, "x");
  check_gpu(q, "q");
  TORCH_CHECK(x.dim() == 2 && q.dim() == 2 && x.size(1) == q.size(1) && q.scalar_type() == at::kChar);
  TORCH_CHECK(scale.numel() == q.size(0));
  if (bias.has_value() && bias->defined())
    TORCH_CHECK(bias->numel() == q.size(0) && bias->scalar_type() == x.scalar_type());
  c10::hip::HIPGuard guard(x.device().index());
  Tensor y = at::empty({x.size(0), q.size(0)}, x.options());
  hip_check(int8_weight_gemm(x.data_ptr(), dt_of(x), q.data_ptr<int8_t>(), scale.data_ptr<float>(),
                             bias.has_value() && bias->defined() ? bias->data_ptr() : nullptr, (int)x.size(0),
                             (int)q.size(0), (int)x.size(1), y.data_ptr(), dt_of(y), cur_stream(x)),
            "int8_weight_gemm");
  return y;
}

// LLM.int8 pieces
Tensor int8_col_outliers_(Tensor x, double threshold) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), "int8_col_outliers: contiguous [M, K]");
  c10::hip::HIPGuard guard(x.device().index());
  Tensor mask = at::empty({x.size(1)}, x.options().dtype(at::kByte));
  Tensor ws = at::empty({x.size(1)}, x.options().dtype(at::kInt));
  hip_check(int8_col_outliers(x.data_ptr(), dt_of16(x), (int)x.size(0), (int)x.size(1), (float)threshold,
                              mask.data_ptr<uint8_t>(), reinterpret_cast<unsigned*>(ws.data_ptr<int32_t>()),
                              cur_stream(x)),
            "int8_col_outliers");
  return mask;
}

std::vector<Tensor> int8_quant_rows_(Tensor x, c10::optional<Tensor> mask) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), "int8_quant_rows: contiguous [M, K]");
  const uint8_t* mp = nullptr;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->scalar_type() == at::kByte && mask->numel() == x.size(1) && mask->is_cuda());
    mp = mask->data_ptr<uint8_t>();
  }
  c10::hip::HIPGuard guard(x.device().index());
  Tensor q = at::empty(x.sizes(), x.options().dtype(at::kChar));
  Tensor s = at::empty({x.size(0)}, x.options().dtype(at::kFloat));
  hip_check(int8_quant_rows(x.data_ptr(), dt_of16(x), (int)x.size(0), (int)x.size(1), mp, q.data_ptr<int8_t>(),
                            s.data_ptr<float>(), cur_stream(x)),
            "int8_quant_rows");
  return {q, s};
}

Tensor int8_mm_(Tensor A, Tensor sa, Tensor B, Tensor sb, c10::optional<Tensor> addend, c10::optional<Tensor> bias,
                const std::string& out_dtype) {
  check_gpu(A, "A");
  check_gpu(B, "B");
  TORCH_CHECK(A.scalar_type() == at::kChar && B.scalar_type() == at::kChar && A.dim() == 2 && B.dim() == 2 &&
                  A.is_contiguous() && B.is_contiguous() && A.size(1) == B.size(1),
              "int8_mm: contiguous int8 A[M,K], B[N,K]");
  const int64_t M = A.size(0), N = B.size(0), K = A.size(1);
  TORCH_CHECK(K % 16 == 0, "int8_mm: K must be a multiple of 16");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(A.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(B.data_ptr()) % 16 == 0,
              "int8_mm: 16-byte aligned operands");
  TORCH_CHECK(sa.scalar_type() == at::kFloat && sa.numel() == M && sb.scalar_type() == at::kFloat && sb.numel() == N);
  const float* ad = nullptr;
  if (addend.has_value() && addend->defined()) {
    TORCH_CHECK(addend->scalar_type() == at::kFloat && addend->is_contiguous() && addend->numel() == M * N);
    ad = addend->data_ptr<float>();
  }
  const void* bp = nullptr;
  int bias_dt = kF32;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->numel() == N && bias->is_contiguous(), "int8_mm: bias [N]");
    bp = bias->data_ptr();
    bias_dt = dt_of16(*bias);
  }
  c10::hip::HIPGuard guard(A.device().index());
  Tensor y = at::empty({M, N}, A.options().dtype(scalar_of(out_dtype)));
  hip_check(int8_mm(A.data_ptr<int8_t>(), sa.data_ptr<float>(), B.data_ptr<int8_t>(), sb.data_ptr<float>(), ad, bp,
                    bias_dt, (int)M, (int)N, (int)K, y.data_ptr(), dt_of16(y), cur_stream(A)),
            "int8_mm");
  return y;
}

std::vector<int64_t> graph_node_census_(int64_t graph) {
  std::vector<int> c(16, 0);
  const int n = graph_node_census(reinterpret_cast<void*>(graph), c.data(), (int)c.size());
  TORCH_CHECK(n >= 0, "graph_node_census: hipGraph query failed");
  std::vector<int64_t> out(c.begin(), c.end());
  out.insert(out.begin(), n);
  return out;  // [total, count of hipGraphNodeType 0, 1, ...]
}

// hipMemsetAsync of a whole tensor (byte value) on the current stream: a capturable memset for the
// graph-editing tests (tests/test_graphs_gpu.py); the framework's own paths issue none
void memset_async_(Tensor t, int64_t value) {
  check_gpu(t, "t");
  TORCH_CHECK(t.is_contiguous(), "memset_async_: contiguous tensor");
  c10::hip::HIPGuard guard(t.device().index());
  hip_check(hipMemsetAsync(t.data_ptr(), (int)value, t.numel() * t.element_size(), cur_stream(t)), "memset_async_");
}

std::vector<std::vector<int64_t>> graph_memset_params_(int64_t graph) {
  std::vector<std::vector<int64_t>> out;
  TORCH_CHECK(graph_memset_params(reinterpret_cast<void*>(graph), &out) >= 0, "graph_memset_params: query failed");
  return out;
}

// a standalone graph with one memset node over t's storage (the runtime's memset-node path alone)
void graph_memset_run_(Tensor t, int64_t value, int64_t esize, int64_t width, int64_t height, int64_t pitch,
                       int64_t reps) {
  check_gpu(t, "t");
  const int64_t rows = height > 0 ? height : 1;
  const int64_t span = (rows - 1) * (pitch > 0 ? pitch : width * esize) + width * esize;
  TORCH_CHECK(esize == 1 || esize == 2 || esize == 4, "graph_memset_run: element size 1, 2 or 4");
  TORCH_CHECK(span <= t.numel() * t.element_size(), "graph_memset_run: the memset exceeds the tensor");
  c10::hip::HIPGuard guard(t.device().index());
  hip_check(graph_memset_run(t.data_ptr(), (uint32_t)value, (int)esize, (size_t)width, (size_t)height,
                             (size_t)pitch, (int)reps, cur_stream(t)),
            "graph_memset_run");
}

int64_t graph_replace_memsets_(int64_t graph) {
  const int r = graph_replace_memsets(reinterpret_cast<void*>(graph));
  TORCH_CHECK(r >= 0, "graph_replace_memsets: hipGraph edit failed");
  return r;
}

// LLM.int8 decode (M <= 32): y = int8 product with outlier columns, two launches, no host sync
// pre-shuffled weights for the decode GEMV (int8_decode.hip): [ceil(N / 16) * 16 * K] int8
Tensor int8_decode_pack_(Tensor q) {
  check_gpu(q, "weight_q");
  TORCH_CHECK(q.dim() == 2 && q.scalar_type() == at::kChar && q.is_contiguous() && q.size(1) % 64 == 0,
              "int8_decode_pack: contiguous int8 [N, K], K % 64 == 0");
  c10::hip::HIPGuard guard(q.device().index());
  const int N = (int)q.size(0), K = (int)q.size(1);
  Tensor p = at::empty({(int64_t)int8_decode_packed_bytes(N, K)}, q.options());
  hip_check(int8_decode_pack(q.data_ptr<int8_t>(), N, K, p.data_ptr<int8_t>(), cur_stream(q)), "int8_decode_pack");
  return p;
}

Tensor int8_decode_(Tensor x, Tensor q, Tensor sw, c10::optional<Tensor> bias, double threshold,
                    const std::string& out_dtype, c10::optional<Tensor> packed) {
  check_gpu(x, "x");
  check_gpu(q, "weight_q");
  TORCH_CHECK(x.dim() == 2 && q.dim() == 2 && q.scalar_type() == at::kChar && x.size(1) == q.size(1),
              "int8_decode: x [M, K], weight_q int8 [N, K]");
  const int64_t M = x.size(0), N = q.size(0), K = x.size(1);
  TORCH_CHECK(int8_decode_supported((int)M, (int)N, (int)K), "int8_decode: M <= 32, K % 64 == 0, K <= ",
              kInt8DecodeMaxK, " (got M=", M, ", K=", K, ")");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(q.data_ptr()) % 16 == 0, "int8_decode: 16-B aligned weight");
  TORCH_CHECK(sw.scalar_type() == at::kFloat && sw.numel() == N && sw.is_contiguous(), "int8_decode: scale [N]");
  const void* bp = nullptr;
  int bias_dt = kF32;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->numel() == N && bias->is_contiguous() && bias->is_cuda(), "int8_decode: bias [N]");
    bp = bias->data_ptr();
    bias_dt = dt_of16(*bias);
  }
  c10::hip::HIPGuard guard(x.device().index());
  if (!x.is_contiguous() || reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 != 0)
    x = x.contiguous().clone();  // the prep kernel reads 16-B chunks
  Tensor ws = at::empty({(int64_t)int8_decode_ws_bytes((int)M, (int)K)}, x.options().dtype(at::kByte));
  Tensor y = at::empty({M, N}, x.options().dtype(scalar_of(out_dtype)));
  const int8_t* wp = nullptr;
  if (packed.has_value() && packed->defined()) {
    TORCH_CHECK(packed->scalar_type() == at::kChar && packed->is_contiguous() && packed->is_cuda() &&
                    packed->numel() == (int64_t)int8_decode_packed_bytes((int)N, (int)K),
                "int8_decode: packed weights from int8_decode_pack");
    wp = packed->data_ptr<int8_t>();
  }
  hip_check(int8_decode(x.data_ptr(), dt_of16(x), (int)M, (int)K, (float)threshold, q.data_ptr<int8_t>(), wp,
                        sw.data_ptr<float>(), bp, bias_dt, (int)N, y.data_ptr(), dt_of16(y), ws.data_ptr(),
                        cur_stream(x)),
            "int8_decode");
  return y;
}

Tensor bn_relu(Tensor x, Tensor scale, Tensor shift, bool relu) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() >= 2);
  const int64_t N = x.size(0), C = x.size(1);
  const int64_t HW = x.numel() / std::max<int64_t>(N * C, 1);
  TORCH_CHECK(scale.numel() == C && shift.numel() == C && scale.scalar_type() == at::kFloat);
  c10::hip::HIPGuard guard(x.device().index());
  Tensor y = at::empty_like(x);
  hip_check(bn_relu_apply(x.data_ptr(), dt_of(x), scale.data_ptr<float>(), shift.data_ptr<float>(), N, C, HW,
                          relu, y.data_ptr(), cur_stream(x)),
            "bn_relu_apply");
  return y;
}

// ------------------------------------------------------------- batchnorm
// Activations as [M, C] rows: NHWC (channels_last-contiguous 4D) or contiguous 2D.
void bn_rows(const Tensor& x, int64_t* M, int* C) {
  TORCH_CHECK(x.is_cuda(), "batchnorm: GPU tensor expected");
  if (x.dim() == 2) {
    TORCH_CHECK(x.is_contiguous(), "batchnorm: 2D input must be contiguous");
  } else {
    TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
                "batchnorm: 4D input must be channels_last-contiguous (NHWC)");
  }
  *C = (int)x.size(1);
  *M = x.numel() / std::max<int64_t>(*C, 1);
  const int V = x.scalar_type() == at::kFloat ? 4 : 8;
  TORCH_CHECK(*C % V == 0, "batchnorm: channels must be a multiple of ", V);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "batchnorm: 16-byte aligned data expected");
}

void same_rows(const Tensor& a, const Tensor& x, const char* name) {
  TORCH_CHECK(a.defined() && a.sizes() == x.sizes() && a.strides() == x.strides() &&
                  a.scalar_type() == x.scalar_type() && a.device() == x.device(),
              "batchnorm: ", name, " must match x (shape, strides, dtype, device)");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(a.data_ptr()) % 16 == 0, "batchnorm: ", name, " not 16-byte aligned");
}

// Ticket array for the last-block hand-off: the caller's (a zeroed int32 tensor
// owned by the BN module, so two modules never share one), else one per device
// created outside graph capture. The kernels re-arm what they use.
int* bn_tickets(const Tensor& x, const c10::optional<Tensor>& given, int need) {
  if (given.has_value() && given->defined()) {
    TORCH_CHECK(given->is_cuda() && given->device() == x.device() && given->scalar_type() == at::kInt &&
                    given->is_contiguous() && given->numel() >= need,
                "batchnorm: tickets must be a zeroed int32 tensor of >= ", need, " elements on x's device");
    return given->data_ptr<int>();
  }
  static std::mutex mu;
  static std::map<int, int*> per_device;
  constexpr int kMax = 1024;
  TORCH_CHECK(need <= kMax, "batchnorm: too many channel tiles");
  std::lock_guard<std::mutex> g(mu);
  const int dev = (int)x.device().index();
  auto it = per_device.find(dev);
  if (it != per_device.end()) return it->second;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  hip_check(hipStreamIsCapturing(cur_stream(x), &st), "hipStreamIsCapturing");
  TORCH_CHECK(st == hipStreamCaptureStatusNone,
              "batchnorm: pass a tickets tensor (ops.norm.BatchNorm2d does) or run once before graph capture");
  int* t = nullptr;
  hip_check(hipMalloc(&t, kMax * sizeof(int)), "hipMalloc(bn tickets)");
  hip_check(hipMemset(t, 0, kMax * sizeof(int)), "hipMemset(bn tickets)");
  per_device[dev] = t;
  return t;
}

const float* opt_f32(const c10::optional<Tensor>& t, int64_t C, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == C,
              "batchnorm: ", name, " must be a contiguous f32 GPU tensor of C elements");
  return t->data_ptr<float>();
}

// Training forward: returns (y, stats[4, C] = mean, invstd, scale, shift).
std::vector<Tensor> bn_fwd_train(Tensor x, c10::optional<Tensor> weight, c10::optional<Tensor> bias,
                                 c10::optional<Tensor> running_mean, c10::optional<Tensor> running_var,
                                 c10::optional<Tensor> num_batches_tracked, c10::optional<Tensor> residual, bool relu,
                                 double momentum, double eps, c10::optional<Tensor> tickets, bool want_mask,
                                 bool stats_only) {
  int64_t M;
  int C;
  bn_rows(x, &M, &C);
  c10::hip::HIPGuard guard(x.device().index());
  BnFwdArgs a{};
  a.x = x.data_ptr();
  if (residual.has_value() && residual->defined()) {
    same_rows(*residual, x, "residual");
    a.residual = residual->data_ptr();
  }
  Tensor y = stats_only ? Tensor() : at::empty_like(x);
  Tensor stats = at::empty({4, C}, x.options().dtype(at::kFloat));
  Tensor ws = at::empty({bn_workspace_floats(M, C, dt_of(x))}, x.options().dtype(at::kFloat));
  a.y = stats_only ? nullptr : y.data_ptr();
  a.dtype = dt_of(x);
  a.M = M;
  a.C = C;
  a.relu = relu ? 1 : 0;
  a.workspace = ws.data_ptr<float>();
  a.tickets = bn_tickets(x, tickets, bn_num_tickets(C, a.dtype));
  a.p.weight = opt_f32(weight, C, "weight");
  a.p.bias = opt_f32(bias, C, "bias");
  a.p.running_mean = const_cast<float*>(opt_f32(running_mean, C, "running_mean"));
  a.p.running_var = const_cast<float*>(opt_f32(running_var, C, "running_var"));
  TORCH_CHECK((a.p.running_mean == nullptr) == (a.p.running_var == nullptr), "batchnorm: running_mean/var together");
  if (num_batches_tracked.has_value() && num_batches_tracked->defined()) {
    TORCH_CHECK(num_batches_tracked->is_cuda() && num_batches_tracked->scalar_type() == at::kLong &&
                num_batches_tracked->numel() == 1, "batchnorm: num_batches_tracked must be a 1-element int64 tensor");
    a.p.num_batches_tracked = num_batches_tracked->data_ptr<int64_t>();
  }
  a.p.momentum = (float)momentum;
  a.p.eps = (float)eps;
  float* st = stats.data_ptr<float>();
  a.p.mean = st;
  a.p.invstd = st + C;
  a.p.scale = st + 2 * C;
  a.p.shift = st + 3 * C;
  Tensor mask;
  if (want_mask && relu && a.residual != nullptr && !stats_only) {  // one byte per 16-B vector of x
    mask = at::empty({M * C / (x.scalar_type() == at::kFloat ? 4 : 8)}, x.options().dtype(at::kByte));
    a.mask_out = mask.data_ptr<uint8_t>();
  }
  hip_check(bn_forward_train(a, cur_stream(x)), "bn_forward_train");
  return {y, stats, mask};
}

// Training forward from precomputed statistics (conv1x1_bn_stats wrote stats = mean, invstd, scale,
// shift and the running statistics): the apply pass only. Returns (y, mask).
std::vector<Tensor> bn_fwd_apply(Tensor x, Tensor stats, c10::optional<Tensor> residual, bool relu, bool want_mask) {
  int64_t M;
  int C;
  bn_rows(x, &M, &C);
  c10::hip::HIPGuard guard(x.device().index());
  TORCH_CHECK(stats.is_cuda() && stats.scalar_type() == at::kFloat && stats.is_contiguous() && stats.numel() == 4 * C,
              "batchnorm: stats must be the [4, C] forward statistics");
  BnFwdArgs a{};
  a.x = x.data_ptr();
  if (residual.has_value() && residual->defined()) {
    same_rows(*residual, x, "residual");
    a.residual = residual->data_ptr();
  }
  Tensor y = at::empty_like(x);
  a.y = y.data_ptr();
  a.dtype = dt_of(x);
  a.M = M;
  a.C = C;
  a.relu = relu ? 1 : 0;
  float* st = stats.data_ptr<float>();
  a.p.mean = st;
  a.p.invstd = st + C;
  a.p.scale = st + 2 * C;
  a.p.shift = st + 3 * C;
  a.stats_ready = 1;
  Tensor mask;
  if (want_mask && relu && a.residual != nullptr) {
    mask = at::empty({M * C / (x.scalar_type() == at::kFloat ? 4 : 8)}, x.options().dtype(at::kByte));
    a.mask_out = mask.data_ptr<uint8_t>();
  }
  hip_check(bn_forward_train(a, cur_stream(x)), "bn_forward_apply");
  return {y, mask};
}

// tile 0: the streaming kernel (conv1x1_bn.hip), else the tiled GEMM's block tile
int64_t conv1x1_bn_num_tickets(int64_t M, int64_t N, int64_t tile, int64_t K) {
  if (tile == 0) return conv1x1_bn_stream_num_tickets((int)M, (int)K, (int)N);
  return gemm_bn_num_tickets((int)M, (int)N, (int)tile);
}

// 1x1 convolution (stride 1) + the training BatchNorm's batch statistics of its output:
// y[M, N] = x[M, K] . w[N, K]^T in bf16 (x: the NHWC activation as rows, w: the [Cout, Cin] weight)
// and stats [4, N] = mean, invstd, scale, shift; running statistics and num_batches_tracked updated.
std::vector<Tensor> conv1x1_bn_stats(Tensor x, Tensor w, c10::optional<Tensor> weight, c10::optional<Tensor> bias,
                                     c10::optional<Tensor> running_mean, c10::optional<Tensor> running_var,
                                     c10::optional<Tensor> num_batches_tracked, double momentum, double eps,
                                     Tensor tickets, int64_t tile) {
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && x.device() == w.device(), "conv1x1_bn_stats: GPU operands");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "conv1x1_bn_stats: x [M, K], w [N, K]");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "conv1x1_bn_stats: bf16");
  TORCH_CHECK(x.stride(1) == 1 && w.stride(1) == 1, "conv1x1_bn_stats: K-contiguous operands");
  TORCH_CHECK(tile == 0 || tile == 128 || tile == 256, "conv1x1_bn_stats: tile 0 (streaming kernel), 128 or 256");
  const int M = (int)x.size(0), N = (int)w.size(0), K = (int)x.size(1);
  TORCH_CHECK(tile != 0 || (conv1x1_bn_stream_supported(K, N) && x.stride(0) == K && w.stride(0) == K),
              "conv1x1_bn_stats: the streaming kernel has no (K, N) = (", K, ", ", N, ") instance");
  TORCH_CHECK(x.size(0) < (1LL << 31) && N % 8 == 0, "conv1x1_bn_stats: N % 8 == 0");
  TORCH_CHECK(gemm_bf16_big_supported(M, N, K, x.stride(0), w.stride(0), x.data_ptr(), w.data_ptr()),
              "conv1x1_bn_stats: K % 64 == 0, 16-B aligned rows");
  c10::hip::HIPGuard guard(x.device().index());
  TORCH_CHECK(tickets.is_cuda() && tickets.device() == x.device() && tickets.scalar_type() == at::kInt &&
                  tickets.is_contiguous() && tickets.numel() >= conv1x1_bn_num_tickets(M, N, tile, K),
              "conv1x1_bn_stats: tickets must be a zeroed int32 tensor of >= ", conv1x1_bn_num_tickets(M, N, tile, K),
              " elements");
  Tensor y = at::empty({M, N}, x.options());
  Tensor stats = at::empty({4, N}, x.options().dtype(at::kFloat));
  Tensor ws = at::empty({tile == 0 ? conv1x1_bn_stream_ws_floats(M, K, N) : gemm_bn_ws_floats(M, N, (int)tile)},
                        x.options().dtype(at::kFloat));
  BigGemmArgs g{};
  g.M = M, g.N = N, g.K = K;
  g.A = x.data_ptr(), g.lda = x.stride(0);
  g.Bt = w.data_ptr(), g.ldb = w.stride(0);
  g.C = y.data_ptr(), g.ldc = N;
  g.out_dtype = kBF16;
  g.alpha = 1.f;
  g.sched = 1;
  g.tile = (int)tile;
  g.split_k = 1;
  GemmBnEpi e{};
  e.ws = ws.data_ptr<float>();
  e.tickets = tickets.data_ptr<int>();
  e.p.weight = opt_f32(weight, N, "weight");
  e.p.bias = opt_f32(bias, N, "bias");
  e.p.running_mean = const_cast<float*>(opt_f32(running_mean, N, "running_mean"));
  e.p.running_var = const_cast<float*>(opt_f32(running_var, N, "running_var"));
  TORCH_CHECK((e.p.running_mean == nullptr) == (e.p.running_var == nullptr), "batchnorm: running_mean/var together");
  if (num_batches_tracked.has_value() && num_batches_tracked->defined()) {
    TORCH_CHECK(num_batches_tracked->is_cuda() && num_batches_tracked->scalar_type() == at::kLong &&
                num_batches_tracked->numel() == 1, "batchnorm: num_batches_tracked must be a 1-element int64 tensor");
    e.p.num_batches_tracked = num_batches_tracked->data_ptr<int64_t>();
  }
  e.p.momentum = (float)momentum;
  e.p.eps = (float)eps;
  float* st = stats.data_ptr<float>();
  e.p.mean = st;
  e.p.invstd = st + N;
  e.p.scale = st + 2 * N;
  e.p.shift = st + 3 * N;
  if (tile == 0)
    hip_check(conv1x1_bn_stream(x.data_ptr(), w.data_ptr(), y.data_ptr(), M, K, N, e, cur_stream(x)),
              "conv1x1_bn_stream");
  else
    hip_check(gemm_bn_stats(g, e, cur_stream(x)), "conv1x1_bn_stats");
  return {y, stats};
}

// Backward: returns (dx, dweight, dbias, dres); dres undefined unless want_dres.
std::vector<Tensor> bn_bwd(Tensor dy, Tensor x, c10::optional<Tensor> y, c10::optional<Tensor> weight, Tensor stats,
                           bool relu, bool want_dres, bool want_dweight, c10::optional<Tensor> tickets,
                           c10::optional<Tensor> dweight_out, c10::optional<Tensor> dbias_out,
                           c10::optional<Tensor> dy2, c10::optional<Tensor> mask) {
  int64_t M;
  int C;
  bn_rows(x, &M, &C);
  same_rows(dy, x, "dy");
  c10::hip::HIPGuard guard(x.device().index());
  TORCH_CHECK(stats.is_cuda() && stats.scalar_type() == at::kFloat && stats.is_contiguous() && stats.numel() == 4 * C,
              "batchnorm: stats must be the [4, C] forward statistics");
  BnBwdArgs a{};
  a.dy = dy.data_ptr();
  if (dy2.has_value() && dy2->defined()) {  // second addend (residual link), same layout as x
    same_rows(*dy2, x, "dy2");
    a.dy2 = dy2->data_ptr();
  }
  a.x = x.data_ptr();
  if (relu && mask.has_value() && mask->defined()) {  // the forward's bit mask (needs want_dres)
    TORCH_CHECK(want_dres && mask->is_cuda() && mask->scalar_type() == at::kByte &&
                    mask->numel() == M * C / (x.scalar_type() == at::kFloat ? 4 : 8),
                "batchnorm: mask must be the forward's [M*C/V] byte mask, with want_dres");
    a.mask = mask->data_ptr<uint8_t>();
  } else if (relu && y.has_value() && y->defined()) {  // else: the mask is recomputed from x (no residual)
    same_rows(*y, x, "y");
    a.y = y->data_ptr();
  }
  Tensor dx = at::empty_like(x);
  Tensor dres = want_dres ? at::empty_like(x) : Tensor();
  Tensor dwb = at::empty({5, C}, x.options().dtype(at::kFloat));  // dweight, dbias, A, B, C
  Tensor ws = at::empty({bn_workspace_floats(M, C, dt_of(x))}, x.options().dtype(at::kFloat));
  a.dx = dx.data_ptr();
  a.dres = want_dres ? dres.data_ptr() : nullptr;
  a.dtype = dt_of(x);
  a.M = M;
  a.C = C;
  a.relu = relu ? 1 : 0;
  a.workspace = ws.data_ptr<float>();
  a.tickets = bn_tickets(x, tickets, bn_num_tickets(C, a.dtype));
  const float* st = stats.data_ptr<float>();
  a.p.weight = opt_f32(weight, C, "weight");
  a.p.mean = st;
  a.p.invstd = st + C;
  a.p.scale = st + 2 * C;
  a.p.shift = st + 3 * C;
  float* d = dwb.data_ptr<float>();
  a.p.dweight = want_dweight ? d : nullptr;
  a.p.dbias = want_dweight ? d + C : nullptr;
  // parameter-gradient destinations given by the caller (DDP bucket slots): written in place
  Tensor dw_out, db_out;
  if (want_dweight && dweight_out.has_value() && dweight_out->defined()) {
    a.p.dweight = const_cast<float*>(opt_f32(dweight_out, C, "dweight_out"));
    dw_out = *dweight_out;
  }
  if (want_dweight && dbias_out.has_value() && dbias_out->defined()) {
    a.p.dbias = const_cast<float*>(opt_f32(dbias_out, C, "dbias_out"));
    db_out = *dbias_out;
  }
  a.p.coef_a = d + 2 * C;
  a.p.coef_b = d + 3 * C;
  a.p.coef_c = d + 4 * C;
  hip_check(bn_backward(a, cur_stream(x)), "bn_backward");
  Tensor dw = want_dweight ? (dw_out.defined() ? dw_out : dwb[0]) : Tensor();
  Tensor db = want_dweight ? (db_out.defined() ? db_out : dwb[1]) : Tensor();
  return {dx, dw, db, dres};
}

// BN backward reduce pass only (for conv1x1_bwd_): returns (g, dweight, dbias, coef[3, C]) where g is the
// masked incoming gradient (ReLU mask, + dy2) and dx = coef[0] g + coef[1] x + coef[2] per channel.
std::vector<Tensor> bn_bwd_reduce(Tensor dy, Tensor x, c10::optional<Tensor> weight, Tensor stats, bool relu,
                                  bool want_dweight, c10::optional<Tensor> tickets, c10::optional<Tensor> dweight_out,
                                  c10::optional<Tensor> dbias_out, c10::optional<Tensor> dy2,
                                  c10::optional<Tensor> mask) {
  int64_t M;
  int C;
  bn_rows(x, &M, &C);
  same_rows(dy, x, "dy");
  c10::hip::HIPGuard guard(x.device().index());
  TORCH_CHECK(stats.is_cuda() && stats.scalar_type() == at::kFloat && stats.is_contiguous() && stats.numel() == 4 * C,
              "batchnorm: stats must be the [4, C] forward statistics");
  BnBwdArgs a{};
  a.dy = dy.data_ptr();
  if (dy2.has_value() && dy2->defined()) {
    same_rows(*dy2, x, "dy2");
    a.dy2 = dy2->data_ptr();
  }
  a.x = x.data_ptr();
  if (relu && mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == at::kByte &&
                    mask->numel() == M * C / (x.scalar_type() == at::kFloat ? 4 : 8),
                "batchnorm: mask must be the forward's [M*C/V] byte mask");
    a.mask = mask->data_ptr<uint8_t>();
  }
  Tensor g = at::empty_like(x);
  Tensor dwb = at::empty({5, C}, x.options().dtype(at::kFloat));
  Tensor ws = at::empty({bn_workspace_floats(M, C, dt_of(x))}, x.options().dtype(at::kFloat));
  a.dx = nullptr;
  a.dres = g.data_ptr();
  a.reduce_only = 1;
  a.dtype = dt_of(x);
  a.M = M;
  a.C = C;
  a.relu = relu ? 1 : 0;
  a.workspace = ws.data_ptr<float>();
  a.tickets = bn_tickets(x, tickets, bn_num_tickets(C, a.dtype));
  const float* st = stats.data_ptr<float>();
  a.p.weight = opt_f32(weight, C, "weight");
  a.p.mean = st;
  a.p.invstd = st + C;
  a.p.scale = st + 2 * C;
  a.p.shift = st + 3 * C;
  float* d = dwb.data_ptr<float>();
  a.p.dweight = want_dweight ? d : nullptr;
  a.p.dbias = want_dweight ? d + C : nullptr;
  Tensor dw_out, db_out;
  if (want_dweight && dweight_out.has_value() && dweight_out->defined()) {
    a.p.dweight = const_cast<float*>(opt_f32(dweight_out, C, "dweight_out"));
    dw_out = *dweight_out;
  }
  if (want_dweight && dbias_out.has_value() && dbias_out->defined()) {
    a.p.dbias = const_cast<float*>(opt_f32(dbias_out, C, "dbias_out"));
    db_out = *dbias_out;
  }
  a.p.coef_a = d + 2 * C;
  a.p.coef_b = d + 3 * C;
  a.p.coef_c = d + 4 * C;
  hip_check(bn_backward(a, cur_stream(x)), "bn_backward(reduce)");
  Tensor dw = want_dweight ? (dw_out.defined() ? dw_out : dwb[0]) : Tensor();
  Tensor db = want_dweight ? (db_out.defined() ? db_out : dwb[1]) : Tensor();
  return {g, dw, db, dwb.narrow(0, 2, 3)};
}

bool conv1x1_bwd_supported_(int64_t K, int64_t N) { return conv1x1_bwd_supported((int)K, (int)N); }

// Backward of BN(conv1x1(x)) from bn_bwd_reduce's (g, coef): returns (dx [M, K], dw [N, K]) in bf16.
std::vector<Tensor> conv1x1_bwd_(Tensor g, Tensor y, Tensor x, Tensor w, Tensor coef) {
  TORCH_CHECK(g.is_cuda() && y.is_cuda() && x.is_cuda() && w.is_cuda() && coef.is_cuda(), "conv1x1_bwd: GPU operands");
  TORCH_CHECK(g.dim() == 2 && y.sizes() == g.sizes() && x.dim() == 2 && w.dim() == 2 && x.size(0) == g.size(0) &&
                  w.size(0) == g.size(1) && w.size(1) == x.size(1),
              "conv1x1_bwd: g, y [M, N], x [M, K], w [N, K]");
  for (const Tensor* t : {&g, &y, &x, &w})
    TORCH_CHECK(t->scalar_type() == at::kBFloat16 && t->is_contiguous(), "conv1x1_bwd: contiguous bf16 operands");
  const int64_t M = g.size(0), N = g.size(1), K = x.size(1);
  TORCH_CHECK(conv1x1_bwd_supported((int)K, (int)N), "conv1x1_bwd: no (K, N) = (", K, ", ", N, ") instance");
  TORCH_CHECK(coef.scalar_type() == at::kFloat && coef.is_contiguous() && coef.numel() == 3 * N,
              "conv1x1_bwd: coef [3, N] float");
  TORCH_CHECK(M < (1LL << 31), "conv1x1_bwd: M < 2^31");
  c10::hip::HIPGuard guard(g.device().index());
  Tensor dx = at::empty({M, K}, x.options());
  Tensor dw = at::empty({N, K}, w.options());
  Tensor ws = at::empty({conv1x1_bwd_ws_floats((int)M, (int)K, (int)N)}, g.options().dtype(at::kFloat));
  hip_check(conv1x1_bwd(g.data_ptr(), y.data_ptr(), x.data_ptr(), w.data_ptr(), coef.data_ptr<float>(), dx.data_ptr(),
                        dw.data_ptr(), ws.data_ptr<float>(), (int)M, (int)K, (int)N,
                        cur_stream(g)),
            "conv1x1_bwd");
  return {dx, dw};
}

// y = ReLU?(x*scale + shift (+ residual)), per channel (eval-mode BN).
Tensor bn_apply_(Tensor x, c10::optional<Tensor> residual, Tensor scale, Tensor shift, bool relu) {
  int64_t M;
  int C;
  bn_rows(x, &M, &C);
  c10::hip::HIPGuard guard(x.device().index());
  const void* r = nullptr;
  if (residual.has_value() && residual->defined()) {
    same_rows(*residual, x, "residual");
    r = residual->data_ptr();
  }
  const float* sc = opt_f32(scale, C, "scale");
  const float* sf = opt_f32(shift, C, "shift");
  Tensor y = at::empty_like(x);
  hip_check(bn_apply(x.data_ptr(), r, y.data_ptr(), dt_of(x), sc, sf, M, C, relu ? 1 : 0, cur_stream(x)), "bn_apply");
  return y;
}

// ------------------------------------------------------------- max pooling (NHWC)
PoolArgs pool_args(const Tensor& x, int64_t Ho, int64_t Wo, std::vector<int64_t> k, std::vector<int64_t> st,
                   std::vector<int64_t> pad) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "maxpool: x must be a channels_last-contiguous 4D GPU tensor");
  TORCH_CHECK(k.size() == 2 && st.size() == 2 && pad.size() == 2, "maxpool: 2D kernel/stride/padding");
  PoolArgs a{};
  a.N = (int)x.size(0); a.C = (int)x.size(1); a.H = (int)x.size(2); a.W = (int)x.size(3);
  a.Ho = (int)Ho; a.Wo = (int)Wo;
  a.kh = (int)k[0]; a.kw = (int)k[1]; a.sh = (int)st[0]; a.sw = (int)st[1]; a.ph = (int)pad[0]; a.pw = (int)pad[1];
  TORCH_CHECK(a.kh >= 1 && a.kw >= 1 && a.kh * a.kw <= 256 && a.sh >= 1 && a.sw >= 1 && a.ph >= 0 && a.pw >= 0 &&
                  2 * a.ph <= a.kh && 2 * a.pw <= a.kw,
              "maxpool: unsupported window");
  TORCH_CHECK((int64_t)(a.H + 2 * a.ph - a.kh) / a.sh + 1 == Ho && (int64_t)(a.W + 2 * a.pw - a.kw) / a.sw + 1 == Wo,
              "maxpool: output size mismatch");
  const int V = x.scalar_type() == at::kFloat ? 4 : 8;
  TORCH_CHECK(a.C % V == 0, "maxpool: channels must be a multiple of ", V);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "maxpool: 16-byte aligned data expected");
  return a;
}

// scale/shift (f32 [C], optional): y = maxpool(ReLU?(x * scale + shift)) -- a training BatchNorm's
// apply pass folded into the pool (ops/norm.bn_relu_maxpool)
std::vector<Tensor> maxpool2d_fwd(Tensor x, std::vector<int64_t> k, std::vector<int64_t> st, std::vector<int64_t> pad,
                                  c10::optional<Tensor> scale, c10::optional<Tensor> shift, bool relu) {
  const int64_t Ho = (x.size(2) + 2 * pad[0] - k[0]) / st[0] + 1, Wo = (x.size(3) + 2 * pad[1] - k[1]) / st[1] + 1;
  PoolArgs a = pool_args(x, Ho, Wo, k, st, pad);
  if (scale.has_value() && scale->defined()) {
    TORCH_CHECK(shift.has_value() && shift->defined(), "maxpool: scale and shift together");
    a.scale = opt_f32(scale, x.size(1), "scale");
    a.shift = opt_f32(shift, x.size(1), "shift");
    a.relu = relu ? 1 : 0;
  }
  c10::hip::HIPGuard guard(x.device().index());
  auto opts = x.options().memory_format(at::MemoryFormat::ChannelsLast);
  Tensor y = at::empty({x.size(0), x.size(1), Ho, Wo}, opts);
  Tensor arg = at::empty({x.size(0), x.size(1), Ho, Wo}, opts.dtype(at::kByte));
  hip_check(maxpool2d_nhwc_forward(x.data_ptr(), y.data_ptr(), arg.data_ptr<uint8_t>(), dt_of(x), a, cur_stream(x)),
            "maxpool2d_nhwc_forward");
  return {y, arg};
}

Tensor maxpool2d_bwd(Tensor gy, Tensor arg, std::vector<int64_t> in_size, std::vector<int64_t> k,
                     std::vector<int64_t> st, std::vector<int64_t> pad) {
  TORCH_CHECK(in_size.size() == 4, "maxpool: input size [N, C, H, W]");
  TORCH_CHECK(gy.is_cuda() && gy.dim() == 4 && gy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  arg.sizes() == gy.sizes() && arg.strides() == gy.strides() && arg.scalar_type() == at::kByte,
              "maxpool backward: gy / argmax must be matching channels_last tensors");
  Tensor gx = at::empty(in_size, gy.options().memory_format(at::MemoryFormat::ChannelsLast));
  PoolArgs a = pool_args(gx, gy.size(2), gy.size(3), k, st, pad);
  c10::hip::HIPGuard guard(gy.device().index());
  hip_check(maxpool2d_nhwc_backward(gy.data_ptr(), arg.data_ptr<uint8_t>(), gx.data_ptr(), dt_of(gy), a,
                                    cur_stream(gy)),
            "maxpool2d_nhwc_backward");
  return gx;
}

// ------------------------------------------------------------- comm
ncclDataType_t nccl_dt(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kChar: return ncclInt8;
    case at::kByte: return ncclUint8;
    default: TORCH_CHECK(false, "RcclComm: unsupported dtype ", t.scalar_type());
  }
  return ncclFloat32;
}

hipStream_t stream_arg(const Tensor& t, int64_t s) {
  return s != 0 ? reinterpret_cast<hipStream_t>(s) : cur_stream(t);
}

}  // namespace
}  // namespace ptdt

PYBIND11_MODULE(_C, m) {
  using namespace ptdt;
  m.doc() = "MI355X-native kernels, RCCL communicator and DDP reducer";
  m.attr("ARCH") = "gfx950";

  m.def("fused_mlp_step", &fused_mlp_step_py, py::arg("X"), py::arg("Yf"), py::arg("Yi"), py::arg("idx"),
        py::arg("P"), py::arg("G"), py::arg("mom"), py::arg("opt_step"), py::arg("loss_out"), py::arg("B"),
        py::arg("Din"), py::arg("H"), py::arg("Dout"), py::arg("loss_kind"), py::arg("ignore_index"),
        py::arg("has_bias"), py::arg("grad_scale"), py::arg("accumulate"), py::arg("update_mode"), py::arg("lr"),
        py::arg("momentum"), py::arg("dampening"), py::arg("weight_decay"), py::arg("nesterov"),
        py::arg("ar") = nullptr);
  m.def("fused_mlp_persistent", &fused_mlp_persistent_py, py::arg("X"), py::arg("Yf"), py::arg("Yi"), py::arg("P"),
        py::arg("G"), py::arg("mom"), py::arg("opt_step"), py::arg("B"), py::arg("Din"), py::arg("H"),
        py::arg("Dout"), py::arg("loss_kind"), py::arg("ignore_index"), py::arg("has_bias"), py::arg("lr"),
        py::arg("momentum"), py::arg("dampening"), py::arg("weight_decay"), py::arg("nesterov"), py::arg("ar"),
        py::arg("n_steps"), py::arg("W"), py::arg("rank"), py::arg("num_samples"), py::arg("shuffle"),
        py::arg("seed"), py::arg("cursor"), py::arg("losses"), py::arg("stamps") = py::none(),
        py::arg("variant") = 0, py::arg("x_zero_padded") = false, py::arg("idx") = py::none(),
        py::arg("cursor_j") = -1);
  py::class_<PersistentPlan, std::shared_ptr<PersistentPlan>>(m, "PersistentPlan")
      .def(py::init<Tensor, c10::optional<Tensor>, c10::optional<Tensor>, Tensor, Tensor, c10::optional<Tensor>,
                    c10::optional<Tensor>, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, bool, double, double,
                    double, double, bool, std::shared_ptr<XgmiComm>, int64_t, int64_t, int64_t, bool, int64_t, Tensor,
                    Tensor, c10::optional<Tensor>, int64_t, bool, c10::optional<Tensor>, c10::optional<Tensor>,
                    int64_t>(),
           py::arg("X"), py::arg("Yf"), py::arg("Yi"), py::arg("P"), py::arg("G"), py::arg("mom"),
           py::arg("opt_step"), py::arg("B"), py::arg("Din"), py::arg("H"), py::arg("Dout"), py::arg("loss_kind"),
           py::arg("ignore_index"), py::arg("has_bias"), py::arg("lr"), py::arg("momentum"), py::arg("dampening"),
           py::arg("weight_decay"), py::arg("nesterov"), py::arg("ar"), py::arg("W"), py::arg("rank"),
           py::arg("num_samples"), py::arg("shuffle"), py::arg("seed"), py::arg("cursor"), py::arg("losses"),
           py::arg("stamps") = py::none(), py::arg("variant") = 0, py::arg("x_zero_padded") = false,
           py::arg("idx") = py::none(), py::arg("lcache") = py::none(), py::arg("idx_e0") = 0)
      .def("launch", &PersistentPlan::launch, py::arg("n_steps"), py::arg("cursor_pos") = -1)
      .def("launch_at", &PersistentPlan::launch_at, py::arg("n_steps"), py::arg("pos"))
      .def_property_readonly("capacity", &PersistentPlan::capacity)
      .def("set_timeline", &PersistentPlan::set_timeline, py::arg("addr"))
      .def("last_launch_ns", &PersistentPlan::last_launch_ns)
      .def("launch_wait_at", &PersistentPlan::launch_wait_at, py::arg("n_steps"), py::arg("pos"), py::arg("mode"),
           py::call_guard<py::gil_scoped_release>());
  py::class_<HostMapped, std::shared_ptr<HostMapped>>(m, "HostMapped")
      .def(py::init<int64_t>(), py::arg("n"))
      .def("zero", &HostMapped::zero)
      .def("read", &HostMapped::read)
      .def("spin", &HostMapped::spin, py::arg("k"), py::arg("timeout_ns"), py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("device_ptr", &HostMapped::device_ptr);
  m.def("clock_calibrate", &clock_calibrate_py, py::arg("n"), py::call_guard<py::gil_scoped_release>());
  m.def("mono_ns", &mono_ns);
  // raw synchronisation primitives with a CLOCK_MONOTONIC return stamp (timeline probes)
  m.def("hip_device_sync_ns", []() {
    hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
    return mono_ns();
  });
  m.def("hip_stream_sync_ns", [](int64_t dev) {
    hip_check(hipStreamSynchronize(c10::hip::getCurrentHIPStream((int)dev).stream()), "hipStreamSynchronize");
    return mono_ns();
  });
  m.def("persistent_engine", &persistent_engine, py::arg("B"), py::arg("Din"), py::arg("H"), py::arg("Dout"),
        py::arg("loss_kind"), py::arg("num_samples"), py::arg("world"), py::arg("variant") = 0,
        py::arg("has_bias") = true);
  m.def("fused_mlp_lds_bytes", [](int B, int Din, int H, int Dout) { return fused_mlp_lds_bytes(B, Din, H, Dout); });
  m.def("sgd_flat_", &sgd_flat_);
  m.def("adam_flat_", &adam_flat_);
  m.def("sgd_multi_", &sgd_multi_, py::arg("ps"), py::arg("gs"), py::arg("moms"), py::arg("step"), py::arg("lr"),
        py::arg("momentum"), py::arg("dampening"), py::arg("wd"), py::arg("nesterov"), py::arg("grad_scale"),
        py::arg("shadows") = std::vector<Tensor>{});
  m.def("adam_multi_", &adam_multi_);
  m.def("bucket_copy", &bucket_copy);
  m.def("scale_", &scale_);
  m.def("cast_multi_", &cast_multi_, py::arg("dsts"), py::arg("srcs"));
  m.def("rgb4_pack", &rgb4_pack_);
  m.def("ce_fwd", &ce_fwd);
  m.def("ce_bwd", &ce_bwd);
  m.def("mse_fwd", &mse_fwd);
  m.def("mse_bwd", &mse_bwd);
  m.def("gemm_", &gemm_, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("bias") = py::none(),
        py::arg("amask") = py::none(), py::arg("relu") = false, py::arg("alpha") = 1.0, py::arg("beta") = 0.0,
        py::arg("colsum") = py::none(), py::arg("split_k") = 1);
  m.def("gemm_big_ok", &gemm_big_ok);
  m.def("gemm_big_", &gemm_big_, py::arg("A"), py::arg("Bt"), py::arg("C"), py::arg("bias") = py::none(),
        py::arg("relu") = false, py::arg("alpha") = 1.0, py::arg("beta") = 0.0, py::arg("sched") = -1,
        py::arg("tile") = 256, py::arg("split_k") = 1);
  m.def("relu_bwd", &relu_bwd);
  m.def("col_sum_", &col_sum_);
  m.def("bn_bwd_reduce", &bn_bwd_reduce, "BN backward reduce pass only: (g, dweight, dbias, coef[3, C])");
  m.def("conv1x1_bwd", &conv1x1_bwd_, "fused BN-apply + 1x1 conv data and weight gradients (bf16)");
  m.def("conv1x1_bwd_supported", &conv1x1_bwd_supported_);
  m.def("graph_node_census", &graph_node_census_, "node count and per-hipGraphNodeType counts of a raw hipGraph_t");
  m.def("memset_async_", &memset_async_, "hipMemsetAsync of a whole tensor (tests of the graph memset rewrite)");
  m.def("graph_memset_params", &graph_memset_params_,
        "memset nodes of a raw hipGraph_t: [dst, value, elementSize, width, height, pitch] each");
  m.def("graph_memset_run", &graph_memset_run_, py::arg("t"), py::arg("value"), py::arg("esize"), py::arg("width"),
        py::arg("height"), py::arg("pitch"), py::arg("reps") = 1);
  m.def("graph_replace_memsets", &graph_replace_memsets_, "replace a raw hipGraph_t's memset nodes by fill-kernel nodes");
  m.def("int8_decode", &int8_decode_, "LLM.int8 decode path (M <= 32): outliers + quantise + int8 GEMV, no host sync",
        py::arg("x"), py::arg("q"), py::arg("sw"), py::arg("bias"), py::arg("threshold"), py::arg("out_dtype"),
        py::arg("packed") = py::none());
  m.def("int8_decode_pack", &int8_decode_pack_, "pre-shuffled int8 weights for the decode GEMV");
  m.def("int8_decode_supported", &int8_decode_supported);
  m.def("sum_all", &sum_all_);
  m.def("philox_", &philox_);
  m.def("one_hot", &one_hot_);
  m.def("gather_rows_", &gather_rows_);
  m.def("device_sampler_", &device_sampler_);
  m.def("quantize_int8", &quantize_int8);
  m.def("int8_linear", &int8_linear);
  m.def("int8_col_outliers", &int8_col_outliers_, py::arg("x"), py::arg("threshold"));
  m.def("int8_quant_rows", &int8_quant_rows_, py::arg("x"), py::arg("mask") = py::none());
  m.def("int8_mm", &int8_mm_, py::arg("A"), py::arg("sa"), py::arg("B"), py::arg("sb"), py::arg("addend") = py::none(),
        py::arg("bias") = py::none(), py::arg("out_dtype") = "float32");
  m.def("bn_relu", &bn_relu);
  m.def("bn_fwd_train", &bn_fwd_train, py::arg("x"), py::arg("weight"), py::arg("bias"), py::arg("running_mean"),
        py::arg("running_var"), py::arg("num_batches_tracked"), py::arg("residual"), py::arg("relu"),
        py::arg("momentum"), py::arg("eps"), py::arg("tickets") = py::none(), py::arg("want_mask") = false,
        py::arg("stats_only") = false);
  m.def("bn_bwd", &bn_bwd, py::arg("dy"), py::arg("x"), py::arg("y"), py::arg("weight"), py::arg("stats"),
        py::arg("relu"), py::arg("want_dres"), py::arg("want_dweight"), py::arg("tickets") = py::none(),
        py::arg("dweight_out") = py::none(), py::arg("dbias_out") = py::none(), py::arg("dy2") = py::none(),
        py::arg("mask") = py::none());
  m.def("maxpool2d_fwd", &maxpool2d_fwd, py::arg("x"), py::arg("k"), py::arg("s"), py::arg("p"),
        py::arg("scale") = py::none(), py::arg("shift") = py::none(), py::arg("relu") = false);
  m.def("maxpool2d_bwd", &maxpool2d_bwd);
  m.def("bn_fwd_apply", &bn_fwd_apply, py::arg("x"), py::arg("stats"), py::arg("residual"), py::arg("relu"),
        py::arg("want_mask"));
  m.def("conv1x1_bn_stats", &conv1x1_bn_stats, py::arg("x"), py::arg("w"), py::arg("weight"), py::arg("bias"),
        py::arg("running_mean"), py::arg("running_var"), py::arg("num_batches_tracked"), py::arg("momentum"),
        py::arg("eps"), py::arg("tickets"), py::arg("tile") = 256);
  m.def("conv1x1_bn_num_tickets", &conv1x1_bn_num_tickets, py::arg("M"), py::arg("N"), py::arg("tile") = 256,
        py::arg("K") = 0);
  m.def("conv1x1_bn_stream_supported", &conv1x1_bn_stream_supported, py::arg("K"), py::arg("N"));
  m.def("bn_apply", &bn_apply_, py::arg("x"), py::arg("residual"), py::arg("scale"), py::arg("shift"),
        py::arg("relu"));

  // A HIP stream restricted to a set of CUs (hipExtStreamCreateWithCUMask), for
  // single-workgroup persistent engines: every launch lands on the same CU, so its
  // code, dataset rows and parameters stay in that XCD's L2 (and the CU's
  // instruction cache) between launches. Returns the raw handle (wrap with
  // torch.cuda.ExternalStream); the stream lives as long as the process.
  // hipSetDeviceFlags before the device's context exists (0 auto, 1 spin, 2 yield,
  // 4 blocking sync): how host waits (hipDeviceSynchronize/events) poll the GPU.
  m.def("set_device_flags", [](int device, unsigned flags) {
    TORCH_CHECK(hipSetDevice(device) == hipSuccess, "hipSetDevice");
    const hipError_t e = hipSetDeviceFlags(flags);
    TORCH_CHECK(e == hipSuccess, "hipSetDeviceFlags: ", hipGetErrorString(e));
  });
  m.def("cu_masked_stream", [](int device, std::vector<int> cus) {
    c10::hip::HIPGuard guard(device);
    int n_cu = 0;
    hip_check(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device), "CU count");
    std::vector<uint32_t> mask((n_cu + 31) / 32, 0u);
    for (int c : cus) {
      TORCH_CHECK(c >= 0 && c < n_cu, "cu_masked_stream: CU ", c, " out of range [0, ", n_cu, ")");
      mask[c / 32] |= 1u << (c % 32);
    }
    hipStream_t st = nullptr;
    hip_check(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()), "hipExtStreamCreateWithCUMask");
    return (uintptr_t)st;
  }, py::arg("device"), py::arg("cus"));
  m.def("torch_perm_", &torch_perm_py, py::arg("seeds"), py::arg("n"), py::arg("W"), py::arg("rank"),
        py::arg("num_samples"), py::arg("out"), py::arg("ws") = py::none());
  m.def("torch_perm_needs_ws", [](int64_t n) { return torch_perm_lds_bytes((int)n) + 624 * 4 > 160 * 1024; });
  m.def("plan_buckets", &plan_buckets);

  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def_static("new_unique_id",
                  []() {
                    auto v = RcclComm::new_unique_id();
                    return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
                  })
      .def(py::init([](int rank, int world, py::bytes uid, int device, double timeout_s, bool fingerprint) {
             std::string s = uid;
             std::vector<uint8_t> v(s.begin(), s.end());
             py::gil_scoped_release nogil;
             return std::make_shared<RcclComm>(rank, world, v, device, timeout_s, fingerprint);
           }),
           py::arg("rank"), py::arg("world"), py::arg("uid"), py::arg("device"), py::arg("timeout_s") = 600.0,
           py::arg("fingerprint") = false)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world", &RcclComm::world)
      .def_property_readonly("device", &RcclComm::device)
      .def_property_readonly("seq", &RcclComm::seq)
      .def("all_reduce",
           [](RcclComm& c, Tensor t, int op, int64_t stream) {
             TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "all_reduce: contiguous GPU tensor");
             c.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dt(t), (ncclRedOp_t)op, stream_arg(t, stream));
           },
           py::arg("t"), py::arg("op") = 0, py::arg("stream") = 0)
      .def("broadcast",
           [](RcclComm& c, Tensor t, int root, int64_t stream) {
             TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "broadcast: contiguous GPU tensor");
             c.broadcast(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dt(t), root, stream_arg(t, stream));
           },
           py::arg("t"), py::arg("root") = 0, py::arg("stream") = 0)
      .def("reduce",
           [](RcclComm& c, Tensor t, int root, int op, int64_t stream) {
             TORCH_CHECK(t.is_cuda() && t.is_contiguous());
             c.reduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dt(t), (ncclRedOp_t)op, root, stream_arg(t, stream));
           },
           py::arg("t"), py::arg("root") = 0, py::arg("op") = 0, py::arg("stream") = 0)
      .def("all_gather",
           [](RcclComm& c, Tensor out, Tensor in, int64_t stream) {
             TORCH_CHECK(out.is_cuda() && in.is_cuda() && out.is_contiguous() && in.is_contiguous());
             TORCH_CHECK(out.numel() == in.numel() * c.world(), "all_gather: out must be world x in");
             c.all_gather(in.data_ptr(), out.data_ptr(), in.numel(), nccl_dt(in), stream_arg(in, stream));
           },
           py::arg("out"), py::arg("inp"), py::arg("stream") = 0)
      .def("reduce_scatter",
           [](RcclComm& c, Tensor out, Tensor in, int op, int64_t stream) {
             TORCH_CHECK(out.is_cuda() && in.is_cuda() && out.is_contiguous() && in.is_contiguous());
             TORCH_CHECK(in.numel() == out.numel() * c.world(), "reduce_scatter: in must be world x out");
             c.reduce_scatter(in.data_ptr(), out.data_ptr(), out.numel(), nccl_dt(in), (ncclRedOp_t)op,
                              stream_arg(in, stream));
           },
           py::arg("out"), py::arg("inp"), py::arg("op") = 0, py::arg("stream") = 0)
      .def("all_to_all",
           [](RcclComm& c, Tensor out, Tensor in, int64_t stream) {
             TORCH_CHECK(out.is_cuda() && in.is_cuda() && out.numel() == in.numel() && in.numel() % c.world() == 0);
             c.all_to_all(in.data_ptr(), out.data_ptr(), in.numel() / c.world(), nccl_dt(in), stream_arg(in, stream));
           },
           py::arg("out"), py::arg("inp"), py::arg("stream") = 0)
      .def("send",
           [](RcclComm& c, Tensor t, int peer, int64_t stream) {
             TORCH_CHECK(t.is_cuda() && t.is_contiguous());
             c.send(t.data_ptr(), t.numel(), nccl_dt(t), peer, stream_arg(t, stream));
           },
           py::arg("t"), py::arg("peer"), py::arg("stream") = 0)
      .def("recv",
           [](RcclComm& c, Tensor t, int peer, int64_t stream) {
             TORCH_CHECK(t.is_cuda() && t.is_contiguous());
             c.recv(t.data_ptr(), t.numel(), nccl_dt(t), peer, stream_arg(t, stream));
           },
           py::arg("t"), py::arg("peer"), py::arg("stream") = 0)
      .def("group_start", &RcclComm::group_start)
      .def("group_end", &RcclComm::group_end)
      .def("error", &RcclComm::error)
      .def("abort", &RcclComm::abort)
      .def_property_readonly("aborted", &RcclComm::aborted)
      .def("fingerprints", &RcclComm::fingerprints)
      .def_property_readonly("captured", &RcclComm::captured)
      .def("expect_captured", &RcclComm::expect_captured, py::arg("k"))
      .def_property_readonly("completed_captured", &RcclComm::completed_captured)
      .def_property_readonly("event_pool_size", &RcclComm::event_pool_size)
      .def_property_readonly("events_created", &RcclComm::events_created);

  py::class_<XgmiComm, std::shared_ptr<XgmiComm>>(m, "XgmiComm")
      .def(py::init<int, int, int, int>(), py::arg("rank"), py::arg("world"), py::arg("max_elems"), py::arg("device"))
      .def("handle", [](XgmiComm& c) { return py::bytes(c.handle()); })
      .def("open", [](XgmiComm& c, std::vector<py::bytes> hs, std::vector<int> devices) {
        std::vector<std::string> v;
        for (auto& h : hs) v.push_back(std::string(h));
        c.open(v, devices);
      }, py::arg("handles"), py::arg("devices") = std::vector<int>{})
      .def_property_readonly("ready", &XgmiComm::ready)
      .def_property_readonly("rank", &XgmiComm::rank)
      .def_property_readonly("world", &XgmiComm::world)
      .def_property_readonly("max_elems", &XgmiComm::max_elems)
      .def_property("max_polls", &XgmiComm::max_polls, &XgmiComm::set_max_polls)
      .def("error", &XgmiComm::error)
      .def("reset_error", &XgmiComm::reset_error)
      .def("all_reduce_avg", [](XgmiComm& c, Tensor t) {
        check_gpu(t, "xgmi all_reduce tensor");
        TORCH_CHECK(t.scalar_type() == at::kFloat, "xgmi all_reduce: fp32");
        TORCH_CHECK(c.ready(), "xgmi all_reduce: communicator not opened");
        TORCH_CHECK(t.numel() <= c.max_elems(), "xgmi all_reduce: tensor larger than the xGMI buffer");
        c10::hip::HIPGuard guard(t.device().index());
        hip_check(xgmi_allreduce_avg(c.args(), t.data_ptr<float>(), (int)t.numel(), cur_stream(t)),
                  "xgmi_allreduce_avg");
      });

  py::class_<RcclClique, std::shared_ptr<RcclClique>>(m, "RcclClique")
      .def(py::init<const std::vector<int>&>())
      .def_property_readonly("size", &RcclClique::size)
      .def("broadcast",
           [](RcclClique& c, std::vector<Tensor> ts, int root) {
             std::vector<void*> b;
             std::vector<hipStream_t> s;
             for (auto& t : ts) {
               b.push_back(t.data_ptr());
               s.push_back(cur_stream(t));
             }
             c.broadcast(b, ts.at(0).numel(), nccl_dt(ts.at(0)), root, s);
           })
      .def("reduce",
           [](RcclClique& c, std::vector<Tensor> ts, int root) {
             std::vector<void*> b;
             std::vector<hipStream_t> s;
             for (auto& t : ts) {
               b.push_back(t.data_ptr());
               s.push_back(cur_stream(t));
             }
             c.reduce(b, ts.at(0).numel(), nccl_dt(ts.at(0)), root, s);
           })
      .def("all_reduce", [](RcclClique& c, std::vector<Tensor> ts) {
        std::vector<void*> b;
        std::vector<hipStream_t> s;
        for (auto& t : ts) {
          b.push_back(t.data_ptr());
          s.push_back(cur_stream(t));
        }
        c.all_reduce(b, ts.at(0).numel(), nccl_dt(ts.at(0)), s);
      });

  py::class_<Reducer, std::shared_ptr<Reducer>>(m, "Reducer")
      .def(py::init([](std::vector<Tensor> params, std::vector<std::vector<int64_t>> buckets,
                       std::shared_ptr<RcclComm> comm, py::object py_allreduce, bool find_unused) {
             Reducer::PyAllReduce fn;
             if (!py_allreduce.is_none()) {
               fn = [py_allreduce](Tensor t) {
                 py::gil_scoped_acquire g;
                 py_allreduce(t);
               };
             }
             return std::make_shared<Reducer>(std::move(params), std::move(buckets), std::move(comm), fn,
                                              find_unused);
           }),
           py::arg("params"), py::arg("buckets"), py::arg("comm"), py::arg("py_allreduce"),
           py::arg("find_unused") = false)
      .def("prepare_for_backward", &Reducer::prepare_for_backward)
      .def("mark_ready", &Reducer::mark_ready)
      .def("finalize", &Reducer::finalize)
      .def("rebuild", &Reducer::rebuild)
      .def("ready_order", &Reducer::ready_order)
      .def("buckets", &Reducer::buckets)
      .def("bucket_tensors", &Reducer::bucket_tensors)
      .def("zero_grads", &Reducer::zero_grads)
      .def("zero_grads_except", &Reducer::zero_grads_except)
      .def("grad_view", &Reducer::grad_view)
      .def_property_readonly("iteration", &Reducer::iteration)
      .def_property_readonly("in_backward", &Reducer::in_backward);
}
