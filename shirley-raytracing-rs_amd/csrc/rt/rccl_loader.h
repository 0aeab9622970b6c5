// rccl_loader.h — RCCL entry points resolved at first use (dlopen), so that libshirley_rt.so loads
// and renders on one GPU where RCCL is absent, and binds to the RCCL copy already in the process when
// there is one (PyTorch-ROCm ships its own librccl.so.1; one RCCL per process, like one HIP runtime).
#pragma once

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <string>

namespace rt {

struct Rccl {
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommInitAll) CommInitAll = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;
  decltype(&ncclGather) Gather = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;  // scene-digest check of rt_render_sharded
  decltype(&ncclAllToAll) AllToAll = nullptr;    // row-band exchange of sample-partitioned frames
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  std::string error;  // why loading failed ("" when every symbol resolved)
  bool ok() const { return error.empty(); }
};

inline Rccl load_rccl() {
  Rccl r;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    const char* e = dlerror();
    r.error = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
    return r;
  }
  auto sym = [&](const char* name) -> void* {
    void* p = dlsym(h, name);
    if (!p && r.error.empty()) r.error = std::string("librccl.so.1 lacks ") + name;
    return p;
  };
  r.GetUniqueId = reinterpret_cast<decltype(r.GetUniqueId)>(sym("ncclGetUniqueId"));
  r.CommInitRank = reinterpret_cast<decltype(r.CommInitRank)>(sym("ncclCommInitRank"));
  r.CommInitAll = reinterpret_cast<decltype(r.CommInitAll)>(sym("ncclCommInitAll"));
  r.CommDestroy = reinterpret_cast<decltype(r.CommDestroy)>(sym("ncclCommDestroy"));
  r.CommGetAsyncError = reinterpret_cast<decltype(r.CommGetAsyncError)>(sym("ncclCommGetAsyncError"));
  r.Gather = reinterpret_cast<decltype(r.Gather)>(sym("ncclGather"));
  r.AllGather = reinterpret_cast<decltype(r.AllGather)>(sym("ncclAllGather"));
  r.AllToAll = reinterpret_cast<decltype(r.AllToAll)>(sym("ncclAllToAll"));
  r.GroupStart = reinterpret_cast<decltype(r.GroupStart)>(sym("ncclGroupStart"));
  r.GroupEnd = reinterpret_cast<decltype(r.GroupEnd)>(sym("ncclGroupEnd"));
  r.GetErrorString = reinterpret_cast<decltype(r.GetErrorString)>(sym("ncclGetErrorString"));
  return r;
}

// The process-wide binding (thread-safe static initialisation).
inline const Rccl& rccl() {
  static const Rccl r = load_rccl();
  return r;
}

}  // namespace rt
