// Host-only checks of the RCCL loader / communicator front end
// (distributed_training_amd/csrc/rccl_comm.cpp), built by
// tests/test_native_build.py with AddressSanitizer + UndefinedBehaviorSanitizer
// on the host code (sanitizers on the host C++ comm layer;
// GPU sanitizers are not available).  Needs no GPU: it exercises dlopen /
// dlsym resolution, the error paths and the unique-id size check.
//
//   usage: rccl_loader_check <path to librccl.so>
#include <cstdio>
#include <stdexcept>
#include <string>

#include "rccl_comm.h"

int main(int argc, char** argv) {
  if (argc < 2) return 64;
  // a missing library is reported, not fatal, and leaves the API unloaded
  std::string e = dta::rccl_load("/nonexistent/librccl.so");
  if (e.empty() || dta::rccl_loaded()) {
    std::printf("FAIL: bad path accepted\n");
    return 2;
  }
  // using the API before a successful load throws
  try {
    (void)dta::rccl_unique_id();
    std::printf("FAIL: unique id without a loaded API\n");
    return 3;
  } catch (const std::runtime_error&) {
  }
  e = dta::rccl_load(argv[1]);
  if (!e.empty() || !dta::rccl_loaded()) {
    std::printf("FAIL: load %s: %s\n", argv[1], e.c_str());
    return 4;
  }
  // loading twice is a no-op
  if (!dta::rccl_load(argv[1]).empty()) return 5;
  int version = 0;
  if (dta::rccl_api().GetVersion(&version) != ncclSuccess || version <= 0) {
    std::printf("FAIL: ncclGetVersion\n");
    return 6;
  }
  if (std::string(dta::rccl_api().GetErrorString(ncclInvalidArgument)).empty()) return 7;
  // a malformed unique id is rejected before any device call
  try {
    dta::RcclComm c(std::string(7, 'x'), 2, 0, 0);
    std::printf("FAIL: short unique id accepted\n");
    return 8;
  } catch (const std::runtime_error&) {
  }
  std::printf("ok rccl %d\n", version);
  return 0;
}
