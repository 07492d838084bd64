// RCCL communicator of the native layer (see comm.h).
#include "comm.h"

#include <dlfcn.h>
#include <link.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <stdexcept>

namespace dtr {

namespace {

// Entry points of the process's (PyTorch's) librccl.  rccl.h supplies only the
// types; every call goes through these pointers, so the extension has no link
// dependency on librccl and can never map a second copy of it.
struct RcclApi {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclCommAbort) abort = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommGetAsyncError) async_error = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::string path;
};

int find_rccl(struct dl_phdr_info* info, size_t, void* data) {
  const char* name = info->dlpi_name;
  if (name && std::strstr(name, "librccl.so")) {
    *static_cast<std::string*>(data) = name;
    return 1;
  }
  return 0;
}

const RcclApi& api() {
  static RcclApi a;
  static std::once_flag once;
  static std::string err;
  std::call_once(once, [] {
    std::string path;
    dl_iterate_phdr(find_rccl, &path);
    void* h = nullptr;
    if (!path.empty()) h = dlopen(path.c_str(), RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) {
      err = "librccl is not loaded in this process (import torch first: the native "
            "communicator reuses PyTorch's RCCL and never loads a second copy)";
      return;
    }
    a.path = path.empty() ? "librccl.so.1" : path;
#define DTR_SYM(field, sym)                                            \
  a.field = reinterpret_cast<decltype(a.field)>(dlsym(h, #sym));       \
  if (!a.field) { err = "librccl lacks " #sym; return; }
    DTR_SYM(get_unique_id, ncclGetUniqueId)
    DTR_SYM(init_rank, ncclCommInitRank)
    DTR_SYM(all_reduce, ncclAllReduce)
    DTR_SYM(broadcast, ncclBroadcast)
    DTR_SYM(abort, ncclCommAbort)
    DTR_SYM(destroy, ncclCommDestroy)
    DTR_SYM(async_error, ncclCommGetAsyncError)
    DTR_SYM(error_string, ncclGetErrorString)
#undef DTR_SYM
  });
  if (!err.empty()) throw std::runtime_error(err);
  return a;
}

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    const RcclApi& a = api();
    throw std::runtime_error(std::string(what) + ": " + a.error_string(r));
  }
}

}  // namespace

struct CommImpl {
  ncclComm_t comm = nullptr;
  bool aborted = false;
};

Comm::Comm(const std::string& id, int world, int rank, int device)
    : impl_(new CommImpl), world_(world), rank_(rank) {
  if (id.size() != NCCL_UNIQUE_ID_BYTES)
    throw std::invalid_argument("Comm: unique id must be NCCL_UNIQUE_ID_BYTES bytes");
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("Comm: bad rank/world");
  const RcclApi& a = api();
  if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("Comm: hipSetDevice failed");
  ncclUniqueId uid;
  std::memcpy(uid.internal, id.data(), NCCL_UNIQUE_ID_BYTES);
  check(a.init_rank(&impl_->comm, world, uid, rank), "ncclCommInitRank");
}

Comm::~Comm() {
  if (impl_ && impl_->comm && !impl_->aborted) {
    try {
      api().destroy(impl_->comm);
    } catch (...) {
    }
  }
}

void Comm::all_reduce(void* buf, size_t count, int dtype, hipStream_t s) const {
  if (impl_->aborted) throw std::runtime_error("all_reduce on an aborted communicator");
  check(api().all_reduce(buf, buf, count, static_cast<ncclDataType_t>(dtype), ncclSum,
                         impl_->comm, s),
        "ncclAllReduce");
}

void Comm::broadcast(void* buf, size_t count, int dtype, int root, hipStream_t s) const {
  if (impl_->aborted) throw std::runtime_error("broadcast on an aborted communicator");
  check(api().broadcast(buf, buf, count, static_cast<ncclDataType_t>(dtype), root, impl_->comm,
                        s),
        "ncclBroadcast");
}

int Comm::async_error() const {
  if (impl_->aborted) return -1;
  ncclResult_t r = ncclSuccess;
  check(api().async_error(impl_->comm, &r), "ncclCommGetAsyncError");
  return static_cast<int>(r);
}

void Comm::abort() {
  if (impl_->comm && !impl_->aborted) {
    impl_->aborted = true;
    api().abort(impl_->comm);
  }
}

std::string Comm::unique_id() {
  ncclUniqueId uid;
  check(api().get_unique_id(&uid), "ncclGetUniqueId");
  return std::string(uid.internal, NCCL_UNIQUE_ID_BYTES);
}

std::string Comm::library() { return api().path; }

}  // namespace dtr
