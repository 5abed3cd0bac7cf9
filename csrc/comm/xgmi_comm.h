// Host side of the xGMI one-shot all-reduce (see xgmi.h): allocates this
// rank's uncached LL buffer, exports / imports IPC handles and owns the
// device-side sequence counter and error flag.
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "xgmi.h"

namespace ptdt {

class XgmiComm {
 public:
  XgmiComm(int rank, int world, int max_elems, int device);
  ~XgmiComm();
  XgmiComm(const XgmiComm&) = delete;
  XgmiComm& operator=(const XgmiComm&) = delete;

  // 64-byte IPC handle of this rank's buffer.
  std::string handle() const;
  // Import every rank's handle (index = rank; own entry ignored). `devices`
  // (optional, index = rank): each rank's device ordinal on this node; a peer on
  // another device this GPU cannot access directly (no xGMI/P2P path) throws, so
  // the caller falls back to RCCL instead of faulting in the first push.
  void open(const std::vector<std::string>& handles, const std::vector<int>& devices = {});
  bool ready() const { return ready_; }
  const XgmiArgs& args() const { return args_; }
  int error() const;  // synchronous read of the device error flag
  void reset_error();
  int rank() const { return args_.rank; }
  int world() const { return args_.world; }
  int max_elems() const { return args_.max_elems; }
  // poll budget of later launches (the self-test runs with the full budget whatever
  // PTDT_XGMI_MAX_POLLS says; fault-injection tests shorten it for the training)
  uint32_t max_polls() const { return args_.max_polls; }
  void set_max_polls(uint32_t n) { args_.max_polls = n == 0u ? 1u : n; }

 private:
  XgmiArgs args_{};
  int device_;
  void* buf_ = nullptr;
  void* ctl_ = nullptr;  // [seq u32 | err i32]
  std::vector<void*> opened_;
  bool ready_ = false;
};

}  // namespace ptdt
