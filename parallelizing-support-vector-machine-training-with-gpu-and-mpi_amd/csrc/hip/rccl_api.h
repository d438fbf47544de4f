// The RCCL entry points the cascade / distributed drivers call, resolved from ONE explicitly loaded
// librccl: the library whose headers this code was compiled against (ROCm's, SVM355_RCCL_PATH), opened
// with RTLD_LOCAL | RTLD_DEEPBIND.  Linking -lrccl instead would bind, inside a PyTorch process, to the
// librccl.so.1 torch had already loaded (its bundled, older copy: 2.26.6 against 2.27.7 headers), so
// the runtime would silently differ from the headers.  SVM355_RCCL_LIB overrides the path.
#pragma once
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <mutex>
#include <stdexcept>
#include <string>

#ifndef SVM355_RCCL_PATH
#define SVM355_RCCL_PATH "/opt/rocm/lib/librccl.so.1"
#endif

namespace svm355 {

struct RcclApi {
  void* handle = nullptr;
  std::string path, error;
  ncclResult_t (*GetVersion)(int*) = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*CommUserRank)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*CommCount)(const ncclComm_t, int*) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Gather)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  bool ok() const { return handle != nullptr; }
};

// Loaded once per process on first use; ok() false (and error set) when the library or a symbol is
// missing -- the callers then fail with that message instead of binding to another RCCL.
inline const RcclApi& rccl() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* env = getenv("SVM355_RCCL_LIB");
    api.path = env && *env ? env : SVM355_RCCL_PATH;
    void* h = dlopen(api.path.c_str(), RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
    if (!h) {
      const char* e = dlerror();
      api.error = "cannot load " + api.path + ": " + (e ? e : "?");
      return;
    }
    bool all = true;
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      if (!fn) {
        all = false;
        api.error += std::string(api.error.empty() ? "" : ", ") + name + " missing in " + api.path;
      }
    };
    sym(api.GetVersion, "ncclGetVersion");
    sym(api.GetUniqueId, "ncclGetUniqueId");
    sym(api.CommInitRank, "ncclCommInitRank");
    sym(api.CommInitAll, "ncclCommInitAll");
    sym(api.CommDestroy, "ncclCommDestroy");
    sym(api.CommAbort, "ncclCommAbort");
    sym(api.CommGetAsyncError, "ncclCommGetAsyncError");
    sym(api.CommUserRank, "ncclCommUserRank");
    sym(api.CommCount, "ncclCommCount");
    sym(api.GetErrorString, "ncclGetErrorString");
    sym(api.Broadcast, "ncclBroadcast");
    sym(api.AllReduce, "ncclAllReduce");
    sym(api.AllGather, "ncclAllGather");
    sym(api.Gather, "ncclGather");
    sym(api.Send, "ncclSend");
    sym(api.Recv, "ncclRecv");
    if (all) api.handle = h;
  });
  return api;
}

// The loaded API or an exception naming what is missing.
inline const RcclApi& rccl_checked() {
  const RcclApi& a = rccl();
  if (!a.ok()) throw std::runtime_error("RCCL: " + a.error);
  return a;
}

}  // namespace svm355
