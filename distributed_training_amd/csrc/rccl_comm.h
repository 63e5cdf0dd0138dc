// Native RCCL communicator (RCCL = ROCm's NCCL-API collective library over
// xGMI / RoCE).  See rccl_comm.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <shared_mutex>
#include <string>

namespace dta {

// Function table resolved with dlopen/dlsym from the librccl.so that PyTorch
// itself loaded, so the process holds exactly one RCCL runtime.
struct RcclApi {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*ReduceScatter)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                                hipStream_t) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  ncclResult_t (*GetVersion)(int*) = nullptr;
  void* handle = nullptr;
};

// Loads the API from `path` (empty: search the already-loaded images).
// Returns an error message, or "" on success.
std::string rccl_load(const std::string& path);
bool rccl_loaded();
const RcclApi& rccl_api();

// Thread safety (the c10d watchdog contract of the reference's init_process_group,
// src/distributed_trainer.py:61-62): a watchdog thread may call abort() while the
// training thread is enqueueing a collective.  Every op holds a SHARED lock on the
// handle for the duration of its ncclXxx call; abort()/destroy() first flag the
// communicator (new calls raise "communicator aborted" without touching it), then
// take the EXCLUSIVE lock, so the handle is released only after every in-flight
// enqueue has returned.  An enqueue stuck inside RCCL (a dead peer during a
// connection setup) would hold its shared lock forever: after `drain_ms` abort()
// calls ncclCommAbort without the lock -- the documented way to unblock such a call
// -- and the handle is left to that call (never destroyed here).
class RcclComm {
 public:
  RcclComm(const std::string& unique_id, int nranks, int rank, int device);
  ~RcclComm();
  void all_reduce(const void* src, void* dst, size_t count, ncclDataType_t dt, ncclRedOp_t op, hipStream_t st);
  void all_gather(const void* src, void* dst, size_t count_per_rank, ncclDataType_t dt, hipStream_t st);
  void reduce_scatter(const void* src, void* dst, size_t count_per_rank, ncclDataType_t dt, ncclRedOp_t op,
                      hipStream_t st);
  void broadcast(const void* src, void* dst, size_t count, ncclDataType_t dt, int root, hipStream_t st);
  void send(const void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t st);
  void recv(void* buf, size_t count, ncclDataType_t dt, int peer, hipStream_t st);
  void group_start();
  void group_end();
  // returns true if every in-flight enqueue drained before the abort
  bool abort(int drain_ms = 10000);
  void destroy();
  bool aborted() const { return aborted_.load(); }
  int rank() const { return rank_; }
  int size() const { return nranks_; }

 private:
  // shared lock on a live handle, or throws "communicator aborted"
  std::shared_lock<std::shared_timed_mutex> use();
  ncclComm_t comm_ = nullptr;
  std::shared_timed_mutex mu_;
  std::atomic<bool> aborted_{false};
  int rank_, nranks_, device_;
};

std::string rccl_unique_id();

}  // namespace dta
