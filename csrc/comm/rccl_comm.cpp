// Native RCCL communicator (see rccl_comm.h for the design notes).
#include "rccl_comm.h"

#include "../kernels/kernels.h"

#include <cstdio>
#include <cstring>
#include <sstream>
#include <stdexcept>

namespace ptdt {

std::string rccl_error_string(ncclResult_t r) { return std::string(ncclGetErrorString(r)); }

static void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

std::vector<uint8_t> RcclComm::new_unique_id() {
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) throw std::runtime_error("ncclGetUniqueId: " + rccl_error_string(r));
  std::vector<uint8_t> out(sizeof(id.internal));
  std::memcpy(out.data(), id.internal, sizeof(id.internal));
  return out;
}

RcclComm::RcclComm(int rank, int world, const std::vector<uint8_t>& uid, int device, double timeout_s,
                   bool fingerprint)
    : rank_(rank), world_(world), device_(device), timeout_s_(timeout_s), fingerprint_(fingerprint) {
  if (uid.size() != sizeof(ncclUniqueId::internal))
    throw std::invalid_argument("RcclComm: unique id must be " +
                                std::to_string(sizeof(ncclUniqueId::internal)) + " bytes");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), uid.size());
  hip_check(hipSetDevice(device), "hipSetDevice");
  check(ncclCommInitRank(&comm_, world, id, rank), "ncclCommInitRank");
  hip_check(hipMalloc(&graph_ctr_dev_, sizeof(uint64_t)), "hipMalloc(graph counter)");
  hip_check(hipMemset(graph_ctr_dev_, 0, sizeof(uint64_t)), "hipMemset(graph counter)");
  void* mirror = nullptr;
  hip_check(hipHostMalloc(&mirror, sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent),
            "hipHostMalloc(graph counter mirror)");
  graph_ctr_host_ = static_cast<volatile uint64_t*>(mirror);
  *graph_ctr_host_ = 0;
  if (timeout_s_ > 0) watchdog_ = std::thread([this] { watchdog_loop(); });
}

RcclComm::~RcclComm() {
  stop_.store(true);
  cv_.notify_all();
  if (watchdog_.joinable()) watchdog_.join();
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& r : pending_)
      if (r.done) (void)hipEventDestroy(r.done);
    pending_.clear();
    for (auto ev : free_events_) (void)hipEventDestroy(ev);
    free_events_.clear();
  }
  if (graph_ctr_dev_) (void)hipFree(graph_ctr_dev_);
  if (graph_ctr_host_) (void)hipHostFree(const_cast<uint64_t*>(graph_ctr_host_));
  if (comm_ != nullptr) {
    if (aborted_.load())
      ; // already aborted by the watchdog
    else
      (void)ncclCommDestroy(comm_);
    comm_ = nullptr;
  }
}

void RcclComm::check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess || r == ncclInProgress) return;
  std::string msg = std::string(what) + " failed on rank " + std::to_string(rank_) + ": " +
                    rccl_error_string(r);
  {
    std::lock_guard<std::mutex> g(mu_);
    if (error_.empty()) error_ = msg;
  }
  throw std::runtime_error(msg);
}

void RcclComm::track(const char* op, size_t count, int dtype, hipStream_t s) {
  if (aborted_.load()) throw std::runtime_error("RcclComm: communicator aborted: " + error());
  const uint64_t seq = seq_.fetch_add(1);
  if (fingerprint_) {
    std::ostringstream os;
    os << seq << ":" << op << ":" << count << ":" << dtype;
    std::lock_guard<std::mutex> g(mu_);
    fp_log_.push_back(os.str());
    if (fp_log_.size() > 4096) fp_log_.erase(fp_log_.begin(), fp_log_.begin() + 2048);
  }
  if (group_depth_ > 0) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(s, &cs);
  if (cs != hipStreamCaptureStatusNone) {
    // part of a graph: a captured counter bump marks its completion at every replay
    hip_check(comm_done_mark(graph_ctr_dev_, const_cast<uint64_t*>(graph_ctr_host_), s), "comm_done_mark");
    captured_.fetch_add(1);
    return;
  }
  if (timeout_s_ <= 0) return;
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!free_events_.empty()) {
      ev = free_events_.back();
      free_events_.pop_back();
    }
  }
  if (ev == nullptr) {
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return;
    events_created_.fetch_add(1);
  }
  if (hipEventRecord(ev, s) != hipSuccess) {
    std::lock_guard<std::mutex> g(mu_);
    free_events_.push_back(ev);
    return;
  }
  std::lock_guard<std::mutex> g(mu_);
  pending_.push_back(CollectiveRecord{seq, op, count, dtype, ev, std::chrono::steady_clock::now()});
}

void RcclComm::expect_captured(uint64_t k) {
  if (k == 0) return;
  std::lock_guard<std::mutex> g(mu_);
  graph_expected_ += k;
  if (timeout_s_ > 0) graph_pending_.emplace_back(graph_expected_, std::chrono::steady_clock::now());
}

uint64_t RcclComm::completed_captured() const { return *graph_ctr_host_; }

size_t RcclComm::event_pool_size() const {
  std::lock_guard<std::mutex> g(mu_);
  return free_events_.size();
}

void RcclComm::watchdog_loop() {
  (void)hipSetDevice(device_);
  // Relaxed capture mode for this thread: its event queries must not
  // invalidate a hipGraph capture running concurrently on the main thread.
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  (void)hipThreadExchangeStreamCaptureMode(&mode);
  std::unique_lock<std::mutex> lk(mu_);
  while (!stop_.load()) {
    cv_.wait_for(lk, std::chrono::milliseconds(100));
    if (stop_.load()) break;
    while (!pending_.empty()) {
      auto& r = pending_.front();
      if (hipEventQuery(r.done) == hipSuccess) {
        free_events_.push_back(r.done);  // recycled: no create/destroy per collective
        pending_.pop_front();
        continue;
      }
      const double age =
          std::chrono::duration<double>(std::chrono::steady_clock::now() - r.issued).count();
      if (age > timeout_s_ && !aborted_.load()) {
        std::ostringstream os;
        os << "watchdog: collective #" << r.seq << " (" << r.op << ", count=" << r.count
           << ") on rank " << rank_ << " did not complete within " << timeout_s_ << " s";
        error_ = os.str();
        std::fprintf(stderr, "[ptdt] %s; aborting communicator\n", error_.c_str());
        aborted_.store(true);
        lk.unlock();
        (void)ncclCommAbort(comm_);
        lk.lock();
      }
      break;
    }
    const uint64_t done = *graph_ctr_host_;
    while (!graph_pending_.empty() && graph_pending_.front().first <= done) graph_pending_.pop_front();
    if (!graph_pending_.empty() && !aborted_.load()) {
      const double age = std::chrono::duration<double>(std::chrono::steady_clock::now() -
                                                       graph_pending_.front().second).count();
      if (age > timeout_s_) {
        std::ostringstream os;
        os << "watchdog: graph-captured collectives on rank " << rank_ << " completed " << done << " of "
           << graph_pending_.front().first << " expected within " << timeout_s_ << " s";
        error_ = os.str();
        std::fprintf(stderr, "[ptdt] %s; aborting communicator\n", error_.c_str());
        aborted_.store(true);
        lk.unlock();
        (void)ncclCommAbort(comm_);
        lk.lock();
      }
    }
    if (!aborted_.load() && comm_ != nullptr) {
      ncclResult_t ae = ncclSuccess;
      lk.unlock();
      (void)ncclCommGetAsyncError(comm_, &ae);
      lk.lock();
      if (ae != ncclSuccess && ae != ncclInProgress) {
        error_ = "async RCCL error on rank " + std::to_string(rank_) + ": " + rccl_error_string(ae);
        std::fprintf(stderr, "[ptdt] %s; aborting communicator\n", error_.c_str());
        aborted_.store(true);
        lk.unlock();
        (void)ncclCommAbort(comm_);
        lk.lock();
      }
    }
  }
}

std::string RcclComm::error() const {
  std::lock_guard<std::mutex> g(mu_);
  return error_;
}

void RcclComm::abort(const std::string& why) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (error_.empty()) error_ = why;
  }
  if (!aborted_.exchange(true) && comm_ != nullptr) (void)ncclCommAbort(comm_);
}

std::vector<std::string> RcclComm::fingerprints() const {
  std::lock_guard<std::mutex> g(mu_);
  return fp_log_;
}

void RcclComm::all_reduce(const void* send, void* recv, size_t count, ncclDataType_t dt,
                          ncclRedOp_t op, hipStream_t s) {
  check(ncclAllReduce(send, recv, count, dt, op, comm_, s), "ncclAllReduce");
  track("all_reduce", count, (int)dt, s);
}

void RcclComm::broadcast(const void* send, void* recv, size_t count, ncclDataType_t dt, int root,
                         hipStream_t s) {
  check(ncclBroadcast(send, recv, count, dt, root, comm_, s), "ncclBroadcast");
  track("broadcast", count, (int)dt, s);
}

void RcclComm::reduce(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                      int root, hipStream_t s) {
  check(ncclReduce(send, recv, count, dt, op, root, comm_, s), "ncclReduce");
  track("reduce", count, (int)dt, s);
}

void RcclComm::all_gather(const void* send, void* recv, size_t send_count, ncclDataType_t dt,
                          hipStream_t s) {
  check(ncclAllGather(send, recv, send_count, dt, comm_, s), "ncclAllGather");
  track("all_gather", send_count, (int)dt, s);
}

void RcclComm::reduce_scatter(const void* send, void* recv, size_t recv_count, ncclDataType_t dt,
                              ncclRedOp_t op, hipStream_t s) {
  check(ncclReduceScatter(send, recv, recv_count, dt, op, comm_, s), "ncclReduceScatter");
  track("reduce_scatter", recv_count, (int)dt, s);
}

void RcclComm::all_to_all(const void* send, void* recv, size_t count_per_peer, ncclDataType_t dt,
                          hipStream_t s) {
  check(ncclAllToAll(send, recv, count_per_peer, dt, comm_, s), "ncclAllToAll");
  track("all_to_all", count_per_peer, (int)dt, s);
}

void RcclComm::send(const void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t s) {
  check(ncclSend(buf, count, dt, peer, comm_, s), "ncclSend");
  track("send", count, (int)dt, s);
}

void RcclComm::recv(void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t s) {
  check(ncclRecv(buf, count, dt, peer, comm_, s), "ncclRecv");
  track("recv", count, (int)dt, s);
}

void RcclComm::group_start() {
  check(ncclGroupStart(), "ncclGroupStart");
  ++group_depth_;
}

void RcclComm::group_end() {
  --group_depth_;
  check(ncclGroupEnd(), "ncclGroupEnd");
}

// ------------------------------------------------------------------ RcclClique
RcclClique::RcclClique(const std::vector<int>& devices) : devices_(devices) {
  comms_.resize(devices.size(), nullptr);
  ncclResult_t r = ncclCommInitAll(comms_.data(), (int)devices.size(), devices.data());
  if (r != ncclSuccess) throw std::runtime_error("ncclCommInitAll: " + rccl_error_string(r));
}

RcclClique::~RcclClique() {
  for (auto c : comms_)
    if (c) (void)ncclCommDestroy(c);
}

static void clique_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + rccl_error_string(r));
}

void RcclClique::broadcast(const std::vector<void*>& bufs, size_t count, ncclDataType_t dt, int root,
                           const std::vector<hipStream_t>& streams) {
  clique_check(ncclGroupStart(), "ncclGroupStart");
  for (size_t i = 0; i < comms_.size(); ++i)
    clique_check(ncclBroadcast(bufs[i], bufs[i], count, dt, root, comms_[i], streams[i]), "ncclBroadcast");
  clique_check(ncclGroupEnd(), "ncclGroupEnd");
}

void RcclClique::reduce(const std::vector<void*>& bufs, size_t count, ncclDataType_t dt, int root,
                        const std::vector<hipStream_t>& streams) {
  clique_check(ncclGroupStart(), "ncclGroupStart");
  for (size_t i = 0; i < comms_.size(); ++i)
    clique_check(ncclReduce(bufs[i], bufs[i], count, dt, ncclSum, root, comms_[i], streams[i]), "ncclReduce");
  clique_check(ncclGroupEnd(), "ncclGroupEnd");
}

void RcclClique::all_reduce(const std::vector<void*>& bufs, size_t count, ncclDataType_t dt,
                            const std::vector<hipStream_t>& streams) {
  clique_check(ncclGroupStart(), "ncclGroupStart");
  for (size_t i = 0; i < comms_.size(); ++i)
    clique_check(ncclAllReduce(bufs[i], bufs[i], count, dt, ncclSum, comms_[i], streams[i]), "ncclAllReduce");
  clique_check(ncclGroupEnd(), "ncclGroupEnd");
}

}  // namespace ptdt
