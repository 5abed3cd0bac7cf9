// Bucketed gradient reducer (see reducer.h).
#include "reducer.h"

#include <cstdlib>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <map>
#include <stdexcept>

#include "../comm/rccl_comm.h"

namespace ptdt {

static ncclDataType_t to_nccl(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    default: throw std::invalid_argument("Reducer: unsupported gradient dtype");
  }
}

static void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("Reducer: ") + what + ": " + hipGetErrorString(e));
}

std::vector<std::vector<int64_t>> plan_buckets(const std::vector<int64_t>& numel,
                                               const std::vector<int64_t>& elem_size,
                                               const std::vector<std::string>& group_key,
                                               const std::vector<int64_t>& order,
                                               int64_t first_cap_bytes, int64_t cap_bytes) {
  // One open bucket per (dtype, device) group, like torch's planner, so params
  // of different groups interleaved in `order` still pack densely.
  std::vector<std::vector<int64_t>> out;
  std::map<std::string, std::pair<std::vector<int64_t>, int64_t>> open;  // key -> (params, bytes)
  std::map<std::string, bool> first_done;
  for (int64_t i : order) {
    const std::string& key = group_key.at(i);
    auto& ob = open[key];
    const int64_t bytes = numel.at(i) * elem_size.at(i);
    ob.first.push_back(i);
    ob.second += bytes;
    const int64_t cap = first_done[key] ? cap_bytes : first_cap_bytes;
    if (ob.second >= cap) {
      out.push_back(std::move(ob.first));
      ob.first.clear();
      ob.second = 0;
      first_done[key] = true;
    }
  }
  for (auto& kv : open)
    if (!kv.second.first.empty()) out.push_back(std::move(kv.second.first));
  return out;
}

Reducer::Reducer(std::vector<at::Tensor> params, std::vector<std::vector<int64_t>> buckets,
                 std::shared_ptr<RcclComm> comm, PyAllReduce py_allreduce, bool find_unused)
    : params_(std::move(params)), comm_(std::move(comm)), py_allreduce_(std::move(py_allreduce)),
      find_unused_(find_unused) {
  if (params_.empty()) throw std::invalid_argument("Reducer: no parameters");
  on_gpu_ = params_[0].is_cuda();
  for (auto& p : params_)
    if (p.is_cuda() != on_gpu_) throw std::invalid_argument("Reducer: mixed CPU/GPU parameters");
  if (on_gpu_) {
    if (!comm_) throw std::invalid_argument("Reducer: GPU parameters need a RcclComm");
    device_ = params_[0].device().index();
    comm_stream_ = c10::hip::getStreamFromPool(/*isHighPriority=*/true, device_);
    // PTDT_FORCE_COLLECTIVE=1: a one-rank job still issues every bucket all-reduce
    // (profiling the overlap on one GPU; the average over one rank is the identity)
    const char* fc = std::getenv("PTDT_FORCE_COLLECTIVE");
    force_collective_ = fc != nullptr && fc[0] == '1';
    hip_ok(hipSetDevice(device_), "hipSetDevice");
    hip_ok(hipEventCreateWithFlags(&ev_ready_, hipEventDisableTiming), "hipEventCreate");
    hip_ok(hipEventCreateWithFlags(&ev_done_, hipEventDisableTiming), "hipEventCreate");
  } else if (!py_allreduce_) {
    throw std::invalid_argument("Reducer: CPU parameters need a Python all-reduce callback");
  }
  param_bucket_.assign(params_.size(), -1);
  param_slot_.assign(params_.size(), -1);
  ready_.assign(params_.size(), 0);
  build(std::move(buckets), /*copy_old=*/true);
}

Reducer::~Reducer() {
  if (ev_ready_) (void)hipEventDestroy(ev_ready_);
  if (ev_done_) (void)hipEventDestroy(ev_done_);
}

void Reducer::build(std::vector<std::vector<int64_t>> plan, bool copy_old) {
  std::vector<char> seen(params_.size(), 0);
  for (auto& b : plan)
    for (int64_t i : b) {
      if (i < 0 || i >= (int64_t)params_.size() || seen[i])
        throw std::invalid_argument("Reducer: bucket plan must be a partition of the parameters");
      seen[i] = 1;
    }
  for (char s : seen)
    if (!s) throw std::invalid_argument("Reducer: bucket plan misses a parameter");

  std::vector<Bucket> nb;
  for (size_t bi = 0; bi < plan.size(); ++bi) {
    Bucket b;
    b.params = plan[bi];
    int64_t off = 0;
    const auto& p0 = params_[b.params[0]];
    for (int64_t i : b.params) {
      if (params_[i].scalar_type() != p0.scalar_type() || params_[i].device() != p0.device())
        throw std::invalid_argument("Reducer: a bucket must hold one dtype on one device");
      b.offsets.push_back(off);
      off += params_[i].numel();
    }
    b.flat = at::zeros({off}, p0.options().requires_grad(false));
    for (size_t k = 0; k < b.params.size(); ++k) {
      const int64_t i = b.params[k];
      auto view = bucket_view(b, k, i);
      const auto& old = params_[i].grad();
      if (copy_old && old.defined()) view.copy_(old);
      param_bucket_[i] = (int64_t)bi;
      param_slot_[i] = (int64_t)k;
      params_[i].mutable_grad() = view;
    }
    nb.push_back(std::move(b));
  }
  buckets_ = std::move(nb);
}

void Reducer::rebuild(std::vector<std::vector<int64_t>> plan) {
  if (in_backward_) throw std::runtime_error("Reducer::rebuild during backward");
  build(std::move(plan), /*copy_old=*/true);
  record_order_ = false;
}

std::vector<std::vector<int64_t>> Reducer::buckets() const {
  std::vector<std::vector<int64_t>> out;
  for (auto& b : buckets_) out.push_back(b.params);
  return out;
}

std::vector<at::Tensor> Reducer::bucket_tensors() const {
  std::vector<at::Tensor> out;
  for (auto& b : buckets_) out.push_back(b.flat);
  return out;
}

void Reducer::zero_grads() {
  for (auto& b : buckets_) b.flat.zero_();
  for (size_t i = 0; i < params_.size(); ++i) ensure_view((int64_t)i);
}

void Reducer::zero_grads_except(const std::vector<int64_t>& skip) {
  std::vector<char> sk(params_.size(), 0);
  for (int64_t i : skip)
    if (i >= 0 && i < (int64_t)params_.size()) sk[i] = 1;
  for (size_t i = 0; i < params_.size(); ++i) {
    if (sk[i]) continue;
    ensure_view((int64_t)i);
    params_[i].mutable_grad().zero_();
  }
}

void Reducer::prepare_for_backward(bool sync) {
  sync_ = sync;
  in_backward_ = true;
  next_launch_ = 0;
  std::fill(ready_.begin(), ready_.end(), 0);
  for (auto& b : buckets_) {
    b.pending = (int64_t)b.params.size();
    b.launched = false;
  }
  if (record_order_) ready_order_.clear();
}

// The grad view of params_[i] inside its bucket. It keeps the parameter's
// strides when the parameter is dense (e.g. channels_last conv weights), so
// grad and param share one memory order ("gradient layout contract") and the
// flat multi-tensor optimizers can treat both as plain arrays.
at::Tensor Reducer::bucket_view(const Bucket& b, size_t k, int64_t i) const {
  const auto& p = params_[i];
  auto flat = b.flat.narrow(0, b.offsets[k], p.numel());
  if (p.is_non_overlapping_and_dense() && !p.is_contiguous()) return flat.as_strided(p.sizes(), p.strides());
  return flat.view(p.sizes());
}

at::Tensor Reducer::grad_view(int64_t i) const {
  if (i < 0 || i >= (int64_t)params_.size()) throw std::out_of_range("Reducer::grad_view");
  return bucket_view(buckets_[param_bucket_[i]], (size_t)param_slot_[i], i);
}

// Make params_[i].grad the bucket view again (a user may have set grads to
// None, or autograd may have assigned a fresh tensor on the first accumulation).
void Reducer::ensure_view(int64_t i) {
  auto& b = buckets_[param_bucket_[i]];
  const int64_t k = param_slot_[i];
  auto view = bucket_view(b, k, i);
  auto& g = params_[i].mutable_grad();
  if (!g.defined()) {
    view.zero_();
    g = view;
  } else if (!g.is_alias_of(view) || g.data_ptr() != view.data_ptr()) {
    view.copy_(g);
    g = view;
  }
}

void Reducer::mark_ready(int64_t i) {
  if (!in_backward_) return;  // a backward that no DDP forward prepared (e.g. eval graph)
  if (i < 0 || i >= (int64_t)params_.size()) throw std::out_of_range("Reducer::mark_ready");
  ensure_view(i);
  if (!sync_) return;  // no_sync(): grads accumulate locally in the bucket views
  if (ready_[i]) {
    throw std::runtime_error(
        "Reducer: parameter " + std::to_string(i) +
        " marked ready twice in one iteration (reused module / multiple backward passes are not "
        "supported with DDP sync; use no_sync() for accumulation)");
  }
  ready_[i] = 1;
  if (record_order_) ready_order_.push_back(i);
  auto& b = buckets_[param_bucket_[i]];
  if (--b.pending == 0) {
    // launch in index order only
    while (next_launch_ < buckets_.size() && buckets_[next_launch_].pending == 0) {
      launch(next_launch_);
      ++next_launch_;
    }
  }
}

void Reducer::launch(size_t bi) {
  auto& b = buckets_[bi];
  b.launched = true;
  if (on_gpu_) {
    if (comm_->world() == 1 && !force_collective_) return;  // the average over one rank is the bucket itself
    hipStream_t compute = c10::hip::getCurrentHIPStream(device_).stream();
    hipStream_t comm = comm_stream_->stream();
    hip_ok(hipEventRecord(ev_ready_, compute), "hipEventRecord");
    hip_ok(hipStreamWaitEvent(comm, ev_ready_, 0), "hipStreamWaitEvent");
    comm_->all_reduce(b.flat.data_ptr(), b.flat.data_ptr(), (size_t)b.flat.numel(),
                      to_nccl(b.flat.scalar_type()), ncclAvg, comm);
  } else {
    py_allreduce_(b.flat);
  }
}

void Reducer::finalize() {
  if (!in_backward_) return;
  in_backward_ = false;
  if (sync_) {
    bool missing = false;
    for (size_t i = 0; i < params_.size(); ++i)
      if (!ready_[i]) missing = true;
    if (missing) {
      if (!find_unused_) {
        std::string names;
        for (size_t i = 0; i < params_.size(); ++i)
          if (!ready_[i]) names += (names.empty() ? "" : ",") + std::to_string(i);
        throw std::runtime_error(
            "Reducer: parameters [" + names +
            "] received no gradient in this iteration. Pass find_unused_parameters=True to the "
            "DDP wrapper if some parameters do not take part in the loss.");
      }
      in_backward_ = true;  // allow mark_ready below
      for (size_t i = 0; i < params_.size(); ++i)
        if (!ready_[i]) {
          auto& g = params_[i].mutable_grad();
          if (!g.defined()) ensure_view((int64_t)i);
          else g.zero_();
          mark_ready((int64_t)i);
        }
      in_backward_ = false;
    }
    if (next_launch_ != buckets_.size())
      throw std::runtime_error("Reducer: internal error, not all buckets launched");
    if (on_gpu_) {
      hipStream_t compute = c10::hip::getCurrentHIPStream(device_).stream();
      hip_ok(hipEventRecord(ev_done_, comm_stream_->stream()), "hipEventRecord");
      hip_ok(hipStreamWaitEvent(compute, ev_done_, 0), "hipStreamWaitEvent");
    }
  }
  ++iteration_;
}

}  // namespace ptdt
