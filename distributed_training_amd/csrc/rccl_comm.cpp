// Native RCCL communicator.
//
// Replaces the reference's implicit c10d ProcessGroupNCCL usage
// (src/distributed_trainer.py:61-62 init_process_group("nccl"); every DDP /
// FSDP collective of src/dist_strategy/*) for the hot path.
// Bootstrap: rank 0 creates the ncclUniqueId, the Python layer ships it to the
// other ranks over torchrun's TCPStore (N03), then ncclCommInitRank.
//
// Collectives are enqueued on a caller-chosen HIP stream and never synchronise
// the host, so they can be overlapped with backward on a dedicated comm stream
// and captured into hipGraphs together with the compute kernels.
#include "rccl_comm.h"

#include <dlfcn.h>

#include <chrono>
#include <cstring>
#include <mutex>
#include <stdexcept>

namespace dta {

static RcclApi g_api;

template <typename F>
static bool sym(void* h, const char* name, F& out) {
  void* p = dlsym(h, name);
  if (!p) return false;
  out = reinterpret_cast<F>(p);
  return true;
}

std::string rccl_load(const std::string& path) {
  if (g_api.handle) return "";
  void* h = path.empty() ? dlopen(nullptr, RTLD_NOW) : dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL);
  if (!h) return std::string("dlopen failed: ") + dlerror();
  bool ok = sym(h, "ncclGetUniqueId", g_api.GetUniqueId) && sym(h, "ncclCommInitRank", g_api.CommInitRank) &&
            sym(h, "ncclCommDestroy", g_api.CommDestroy) && sym(h, "ncclCommAbort", g_api.CommAbort) &&
            sym(h, "ncclAllReduce", g_api.AllReduce) && sym(h, "ncclAllGather", g_api.AllGather) &&
            sym(h, "ncclReduceScatter", g_api.ReduceScatter) && sym(h, "ncclBroadcast", g_api.Broadcast) &&
            sym(h, "ncclSend", g_api.Send) && sym(h, "ncclRecv", g_api.Recv) &&
            sym(h, "ncclGroupStart", g_api.GroupStart) && sym(h, "ncclGroupEnd", g_api.GroupEnd) &&
            sym(h, "ncclGetErrorString", g_api.GetErrorString) && sym(h, "ncclGetVersion", g_api.GetVersion);
  if (!ok) return "librccl is missing required ncclXxx symbols";
  g_api.handle = h;
  return "";
}

bool rccl_loaded() { return g_api.handle != nullptr; }
const RcclApi& rccl_api() { return g_api; }

static void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    std::string msg = std::string("RCCL ") + what + " failed: " +
                      (g_api.GetErrorString ? g_api.GetErrorString(r) : "unknown");
    throw std::runtime_error(msg);
  }
}

static void need_api() {
  if (!g_api.handle) throw std::runtime_error("RCCL API not loaded (call rccl_load first)");
}

std::string rccl_unique_id() {
  need_api();
  ncclUniqueId id;
  check(g_api.GetUniqueId(&id), "ncclGetUniqueId");
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

RcclComm::RcclComm(const std::string& unique_id, int nranks, int rank, int device)
    : rank_(rank), nranks_(nranks), device_(device) {
  need_api();
  if (unique_id.size() != sizeof(ncclUniqueId)) throw std::runtime_error("bad ncclUniqueId size");
  ncclUniqueId id;
  std::memcpy(&id, unique_id.data(), sizeof(id));
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("hipSetDevice failed");
  check(g_api.CommInitRank(&comm_, nranks, id, rank), "ncclCommInitRank");
}

RcclComm::~RcclComm() { destroy(); }

std::shared_lock<std::shared_timed_mutex> RcclComm::use() {
  std::shared_lock<std::shared_timed_mutex> lk(mu_);
  if (aborted_.load() || comm_ == nullptr) throw std::runtime_error("RCCL communicator aborted");
  return lk;
}

bool RcclComm::abort(int drain_ms) {
  if (aborted_.exchange(true)) return true;  // (a second abort: the first one owns the handle)
  std::unique_lock<std::shared_timed_mutex> lk(mu_, std::defer_lock);
  const bool drained = lk.try_lock_for(std::chrono::milliseconds(drain_ms > 0 ? drain_ms : 0));
  ncclComm_t c = comm_;
  if (c) g_api.CommAbort(c);
  if (drained) comm_ = nullptr;  // else the stuck call still references it: leaked, never freed twice
  return drained;
}

void RcclComm::destroy() {
  if (aborted_.exchange(true)) return;
  std::unique_lock<std::shared_timed_mutex> lk(mu_);
  if (comm_ && g_api.CommDestroy) g_api.CommDestroy(comm_);
  comm_ = nullptr;
}

void RcclComm::all_reduce(const void* src, void* dst, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                          hipStream_t st) {
  auto lk = use();
  check(g_api.AllReduce(src, dst, count, dt, op, comm_, st), "ncclAllReduce");
}
void RcclComm::all_gather(const void* src, void* dst, size_t count, ncclDataType_t dt, hipStream_t st) {
  auto lk = use();
  check(g_api.AllGather(src, dst, count, dt, comm_, st), "ncclAllGather");
}
void RcclComm::reduce_scatter(const void* src, void* dst, size_t count, ncclDataType_t dt, ncclRedOp_t op,
                              hipStream_t st) {
  auto lk = use();
  check(g_api.ReduceScatter(src, dst, count, dt, op, comm_, st), "ncclReduceScatter");
}
void RcclComm::broadcast(const void* src, void* dst, size_t count, ncclDataType_t dt, int root, hipStream_t st) {
  auto lk = use();
  check(g_api.Broadcast(src, dst, count, dt, root, comm_, st), "ncclBroadcast");
}
void RcclComm::send(const void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t st) {
  auto lk = use();
  check(g_api.Send(buf, count, dt, peer, comm_, st), "ncclSend");
}
void RcclComm::recv(void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t st) {
  auto lk = use();
  check(g_api.Recv(buf, count, dt, peer, comm_, st), "ncclRecv");
}
void RcclComm::group_start() {
  auto lk = use();
  check(g_api.GroupStart(), "ncclGroupStart");
}
void RcclComm::group_end() {
  auto lk = use();
  check(g_api.GroupEnd(), "ncclGroupEnd");
}

}  // namespace dta
