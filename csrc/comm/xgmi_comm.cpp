// Host side of the xGMI one-shot all-reduce (see xgmi_comm.h / xgmi.h).
#include "xgmi_comm.h"

#include <algorithm>
#include <cstdlib>

#include <cstring>
#include <stdexcept>

namespace ptdt {

static void ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("XgmiComm: ") + what + ": " + hipGetErrorString(e));
}

XgmiComm::XgmiComm(int rank, int world, int max_elems, int device) : device_(device) {
  if (world < 1 || world > kXgmiMaxRanks || rank < 0 || rank >= world || max_elems <= 0 ||
      (int64_t)2 * world * max_elems >= (int64_t)1 << 31)  // device slot offsets are 32-bit
    throw std::invalid_argument("XgmiComm: bad rank/world/max_elems");
  ok(hipSetDevice(device), "hipSetDevice");
  const size_t bytes = (size_t)2 * world * max_elems * sizeof(uint64_t);
  // uncached: remote xGMI stores must be visible to this GPU's polls (no stale L2 lines)
  ok(hipExtMallocWithFlags(&buf_, bytes, hipDeviceMallocUncached), "hipExtMallocWithFlags(uncached)");
  ok(hipMemset(buf_, 0, bytes), "hipMemset");
  ok(hipMalloc(&ctl_, 64), "hipMalloc");
  ok(hipMemset(ctl_, 0, 64), "hipMemset");
  ok(hipDeviceSynchronize(), "hipDeviceSynchronize");
  args_.local = static_cast<uint64_t*>(buf_);
  for (auto& p : args_.peers) p = nullptr;
  args_.peers[rank] = args_.local;
  args_.seq = static_cast<uint32_t*>(ctl_);
  args_.err = reinterpret_cast<int*>(static_cast<char*>(ctl_) + 4);
  args_.rank = rank;
  args_.world = world;
  args_.max_elems = max_elems;
  args_.max_polls = kXgmiMaxPolls;
  if (const char* v = std::getenv("PTDT_XGMI_MAX_POLLS")) {  // shorter bound for fault-injection tests
    const long n = std::strtol(v, nullptr, 10);
    if (n > 0) args_.max_polls = (uint32_t)std::min<long>(n, (long)kXgmiMaxPolls);
  }
  args_.drop_push = 0u;
  args_.flags = kXgmiPair;
  if (const char* v = std::getenv("PTDT_XGMI_PAIR")) {
    if (std::strtol(v, nullptr, 10) == 0) args_.flags &= ~kXgmiPair;
  }
  if (const char* v = std::getenv("PTDT_FAULT_XGMI_DROP_RANK")) {
    if (std::strtol(v, nullptr, 10) == rank) {
      const char* sq = std::getenv("PTDT_FAULT_XGMI_DROP_SEQ");
      const long s0 = sq ? std::strtol(sq, nullptr, 10) : 64;  // after the self-test's collectives
      args_.drop_push = (uint32_t)(s0 > 0 ? s0 : 1);
    }
  }
  if (world == 1) ready_ = true;
}

XgmiComm::~XgmiComm() {
  (void)hipSetDevice(device_);
  (void)hipDeviceSynchronize();
  for (void* p : opened_) (void)hipIpcCloseMemHandle(p);
  if (buf_) (void)hipFree(buf_);
  if (ctl_) (void)hipFree(ctl_);
}

std::string XgmiComm::handle() const {
  hipIpcMemHandle_t h;
  ok(hipIpcGetMemHandle(&h, buf_), "hipIpcGetMemHandle");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void XgmiComm::open(const std::vector<std::string>& handles, const std::vector<int>& devices) {
  if ((int)handles.size() != args_.world) throw std::invalid_argument("XgmiComm::open: need one handle per rank");
  if (!devices.empty() && (int)devices.size() != args_.world)
    throw std::invalid_argument("XgmiComm::open: need one device ordinal per rank");
  ok(hipSetDevice(device_), "hipSetDevice");
  for (int p = 0; p < args_.world; ++p) {
    if (p == args_.rank || devices.empty() || devices[p] == device_) continue;
    int can = 0;
    ok(hipDeviceCanAccessPeer(&can, device_, devices[p]), "hipDeviceCanAccessPeer");
    if (!can)
      throw std::runtime_error("XgmiComm::open: device " + std::to_string(device_) + " cannot access peer device " +
                               std::to_string(devices[p]));
  }
  for (int p = 0; p < args_.world; ++p) {
    if (p == args_.rank) continue;
    if (handles[p].size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("XgmiComm::open: bad handle");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[p].data(), sizeof(h));
    void* ptr = nullptr;
    ok(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    opened_.push_back(ptr);
    args_.peers[p] = static_cast<uint64_t*>(ptr);
  }
  ready_ = true;
}

int XgmiComm::error() const {
  int e = 0;
  ok(hipMemcpy(&e, args_.err, sizeof(int), hipMemcpyDeviceToHost), "hipMemcpy");
  return e;
}

void XgmiComm::reset_error() { ok(hipMemset(args_.err, 0, sizeof(int)), "hipMemset"); }

}  // namespace ptdt
