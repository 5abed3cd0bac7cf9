// Bucketed gradient reducer for DistributedDataParallel (C++).
//
// Reference: DistributedDataParallel(model, device_ids=[gpu_id]) ddp_gpus.py:32
// builds torch's C++ Reducer: reverse-order bucket planning
// (1 MiB first bucket, 25 MiB cap), per-grad autograd hooks that copy grads
// into a flat bucket scaled by 1/world_size, an all-reduce per full bucket and
// a finalize that waits and copies back.
//
// This reducer is designed for MI355X instead:
//   * buckets are the .grad storage (every parameter's .grad is a view into its
//     bucket), so there is no per-step pack/unpack copy;
//   * the average is done by RCCL itself (ncclAvg) -- no scale kernel;
//   * bucket caps default to xGMI-friendly sizes (small first bucket to shorten
//     the post-backward tail, large caps so each of the 7 links gets >> 1 MB per
//     ring step; see parallel/bucketing.py for the sizing rule);
//   * all-reduces run on a dedicated high-priority comm stream, ordered after
//     the producing backward kernels by an event, overlapping the remaining
//     backward; finalize joins the comm stream back into the compute stream;
//   * buckets are launched strictly in index order on every rank (a bucket that
//     becomes ready early waits for its predecessors), so collective order is
//     identical across ranks even if autograd's ready order differs;
//   * after the first iteration the buckets can be rebuilt in the observed
//     gradient-ready order (rank 0's order, broadcast by the Python layer).
// The same C++ class drives CPU tensors (tests, gloo) through a Python
// all-reduce callback, so the CPU plumbing tests exercise this exact code.
#pragma once

#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>

#include <functional>
#include <memory>
#include <optional>
#include <string>
#include <vector>

namespace ptdt {

class RcclComm;

// Plan buckets: walk `order` (parameter indices), start a new bucket when the
// dtype/device changes or the byte cap would be exceeded. The first bucket uses
// `first_cap_bytes`, later ones `cap_bytes`.
std::vector<std::vector<int64_t>> plan_buckets(const std::vector<int64_t>& numel,
                                               const std::vector<int64_t>& elem_size,
                                               const std::vector<std::string>& group_key,
                                               const std::vector<int64_t>& order,
                                               int64_t first_cap_bytes, int64_t cap_bytes);

class Reducer {
 public:
  using PyAllReduce = std::function<void(at::Tensor)>;  // in-place average (CPU path)

  Reducer(std::vector<at::Tensor> params, std::vector<std::vector<int64_t>> buckets,
          std::shared_ptr<RcclComm> comm, PyAllReduce py_allreduce, bool find_unused);
  ~Reducer();

  // Called by the DDP forward: starts a new iteration.
  void prepare_for_backward(bool sync);
  // Called from each parameter's post-accumulate-grad hook.
  void mark_ready(int64_t param_index);
  // Called once at the end of backward (autograd engine callback).
  void finalize();
  // Re-plan buckets (e.g. in rank 0's observed ready order).
  void rebuild(std::vector<std::vector<int64_t>> buckets);

  std::vector<int64_t> ready_order() const { return ready_order_; }
  std::vector<std::vector<int64_t>> buckets() const;
  std::vector<at::Tensor> bucket_tensors() const;
  int64_t iteration() const { return iteration_; }
  bool in_backward() const { return in_backward_; }
  void zero_grads();
  // Zero only the slots of the parameters NOT in `skip` (their .grad re-bound to the views): the
  // skipped ones are grad-sink parameters whose producer overwrites the whole slot every backward.
  void zero_grads_except(const std::vector<int64_t>& skip);
  // A fresh view of parameter i's slot in its bucket (the parameter's own strides):
  // autograd "steals" it as .grad when a cast's backward writes the gradient straight
  // into it (ops/conv.py grad sinks), so no separate accumulate kernel runs.
  at::Tensor grad_view(int64_t i) const;

 private:
  struct Bucket {
    std::vector<int64_t> params;
    std::vector<int64_t> offsets;  // element offsets in flat
    at::Tensor flat;
    int64_t pending = 0;
    bool launched = false;
  };
  void build(std::vector<std::vector<int64_t>> buckets, bool copy_old);
  void launch(size_t b);
  void ensure_view(int64_t i);
  at::Tensor bucket_view(const Bucket& b, size_t k, int64_t i) const;

  std::vector<at::Tensor> params_;
  std::vector<Bucket> buckets_;
  std::vector<int64_t> param_bucket_;
  std::vector<int64_t> param_slot_;
  std::vector<char> ready_;
  std::vector<int64_t> ready_order_;
  std::shared_ptr<RcclComm> comm_;
  PyAllReduce py_allreduce_;
  bool find_unused_;
  bool on_gpu_ = false;
  bool sync_ = true;
  bool in_backward_ = false;
  bool record_order_ = true;
  size_t next_launch_ = 0;
  int64_t iteration_ = 0;
  std::optional<c10::hip::HIPStream> comm_stream_;
  hipEvent_t ev_ready_ = nullptr;  // compute -> comm ordering
  hipEvent_t ev_done_ = nullptr;   // comm -> compute join
  bool force_collective_ = false;  // PTDT_FORCE_COLLECTIVE=1: collectives even at world 1
  int device_ = -1;
};

}  // namespace ptdt
