// Native RCCL communicator (see rccl_comm.h for the design notes).
#include "rccl_comm.h"

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
  }
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
  if (timeout_s_ <= 0 || group_depth_ > 0) return;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(s, &cs);
  if (cs != hipStreamCaptureStatusNone) return;  // replayed later; not tracked
  hipEvent_t ev = nullptr;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return;
  if (hipEventRecord(ev, s) != hipSuccess) {
    (void)hipEventDestroy(ev);
    return;
  }
  std::lock_guard<std::mutex> g(mu_);
  pending_.push_back(CollectiveRecord{seq, op, count, dtype, ev, std::chrono::steady_clock::now()});
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
        (void)hipEventDestroy(r.done);
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
