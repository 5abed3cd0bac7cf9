// Native RCCL communicator for MI355X (one process per GPU over xGMI, or one
// process driving several GPUs for the single-process DataParallel path).
//
// Reference mapping: the reference relies on
// c10d ProcessGroupNCCL (init_process_group("nccl"), ddp_gpus.py:16), the DDP
// reducer's all-reduce, torch.cuda.nccl.reduce / broadcast_coalesced for
// nn.DataParallel, and CUDA peer copies for model parallel. This layer gives
// the framework its own communicator on top of RCCL:
//   * unique-id exchange through the c10d TCPStore (done by the Python side,
//     which passes the 128-byte id in), ncclCommInitRank per rank;
//   * collectives enqueued on a caller-chosen HIP stream (so they can be
//     captured into hipGraphs and overlapped on a dedicated comm stream);
//   * a watchdog thread that polls ncclCommGetAsyncError and the completion
//     events of outstanding collectives and aborts the communicator on error
//     or timeout instead of hanging;
//   * an optional collective fingerprint log (op, count, dtype, seq#) for
//     cross-rank mismatch detection;
//   * completion tracking without per-call allocation: eager collectives take
//     a recycled event from a pool; a collective issued under hipGraph capture
//     is followed (in the graph) by a one-thread kernel that bumps a device
//     counter and mirrors it into host-mapped memory, so replays are watched
//     too -- the replaying code declares how many completions it expects
//     (expect_captured) and the watchdog polls the mirror.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace ptdt {

std::string rccl_error_string(ncclResult_t r);

struct CollectiveRecord {
  uint64_t seq;
  std::string op;
  size_t count;
  int dtype;
  hipEvent_t done;  // nullptr when issued under stream capture
  std::chrono::steady_clock::time_point issued;
};

class RcclComm {
 public:
  static std::vector<uint8_t> new_unique_id();

  // Multi-process: this process is `rank` of `world` on HIP device `device`.
  RcclComm(int rank, int world, const std::vector<uint8_t>& uid, int device, double timeout_s,
           bool fingerprint);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }

  // op: 0 sum, 1 prod, 2 max, 3 min, 4 avg (ncclRedOp_t values)
  void all_reduce(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                  hipStream_t s);
  void broadcast(const void* send, void* recv, size_t count, ncclDataType_t dt, int root, hipStream_t s);
  void reduce(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclRedOp_t op, int root,
              hipStream_t s);
  void all_gather(const void* send, void* recv, size_t send_count, ncclDataType_t dt, hipStream_t s);
  void reduce_scatter(const void* send, void* recv, size_t recv_count, ncclDataType_t dt,
                      ncclRedOp_t op, hipStream_t s);
  void all_to_all(const void* send, void* recv, size_t count_per_peer, ncclDataType_t dt, hipStream_t s);
  void send(const void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t s);
  void recv(void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t s);
  void group_start();
  void group_end();

  // Error state: non-empty after the watchdog detected an async error/timeout.
  std::string error() const;
  void abort(const std::string& why);
  bool aborted() const { return aborted_.load(); }
  uint64_t seq() const { return seq_.load(); }
  std::vector<std::string> fingerprints() const;

  // hipGraph-captured collectives: `captured()` counts the collectives captured
  // so far (a graph's share is the difference around its capture); after each
  // replay of a graph holding k of them call expect_captured(k). completed_captured()
  // is the device counter's host mirror.
  uint64_t captured() const { return captured_.load(); }
  void expect_captured(uint64_t k);
  uint64_t completed_captured() const;
  size_t event_pool_size() const;
  size_t events_created() const { return events_created_.load(); }

 private:
  void check(ncclResult_t r, const char* what);
  void track(const char* op, size_t count, int dtype, hipStream_t s);
  void watchdog_loop();

  int rank_, world_, device_;
  ncclComm_t comm_ = nullptr;
  double timeout_s_;
  bool fingerprint_;
  std::atomic<uint64_t> seq_{0};
  std::atomic<bool> aborted_{false};
  std::atomic<bool> stop_{false};
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<CollectiveRecord> pending_;
  std::vector<hipEvent_t> free_events_;  // recycled completion events
  std::atomic<size_t> events_created_{0};
  uint64_t* graph_ctr_dev_ = nullptr;              // device counter (captured kernels bump it)
  volatile uint64_t* graph_ctr_host_ = nullptr;    // host-mapped mirror read by the watchdog
  std::atomic<uint64_t> captured_{0};
  uint64_t graph_expected_ = 0;
  std::deque<std::pair<uint64_t, std::chrono::steady_clock::time_point>> graph_pending_;
  std::vector<std::string> fp_log_;
  std::string error_;
  std::thread watchdog_;
  int group_depth_ = 0;
};

// Single process, several devices (nn.DataParallel replacement): one RCCL
// communicator per device created with ncclCommInitAll; every collective is a
// grouped call with one stream per device.
class RcclClique {
 public:
  explicit RcclClique(const std::vector<int>& devices);
  ~RcclClique();
  int size() const { return (int)comms_.size(); }
  const std::vector<int>& devices() const { return devices_; }
  // buffers[i] lives on devices[i]; streams[i] on that device
  void broadcast(const std::vector<void*>& bufs, size_t count, ncclDataType_t dt, int root,
                 const std::vector<hipStream_t>& streams);
  void reduce(const std::vector<void*>& bufs, size_t count, ncclDataType_t dt, int root,
              const std::vector<hipStream_t>& streams);
  void all_reduce(const std::vector<void*>& bufs, size_t count, ncclDataType_t dt,
                  const std::vector<hipStream_t>& streams);

 private:
  std::vector<int> devices_;
  std::vector<ncclComm_t> comms_;
};

}  // namespace ptdt
