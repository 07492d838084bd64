// Communicator of the native layer (see comm.h): the Comm front end, the RCCL
// transport and the loopback diagnostics transport.  The shared-memory
// rehearsal transport lives in comm_shm.cpp.
#include "comm.h"

#include <dlfcn.h>
#include <link.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstring>
#include <mutex>
#include <stdexcept>

namespace dtr {

size_t comm_dtype_bytes(int dtype) {
  switch (dtype) {
    case COMM_F32: return 4;
    case COMM_BF16: return 2;
    case COMM_F64: return 8;
    case COMM_I64: return 8;
    default: throw std::invalid_argument("comm: unsupported dtype code " + std::to_string(dtype));
  }
}

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
  decltype(&ncclGetVersion) get_version = nullptr;   // optional (reporting only)
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
    a.get_version = reinterpret_cast<decltype(a.get_version)>(dlsym(h, "ncclGetVersion"));
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

class RcclTransport final : public Transport {
 public:
  RcclTransport(const std::string& id, int world, int rank, int device) {
    if (id.size() != NCCL_UNIQUE_ID_BYTES)
      throw std::invalid_argument("Comm: unique id must be NCCL_UNIQUE_ID_BYTES bytes");
    const RcclApi& a = api();
    if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("Comm: hipSetDevice failed");
    ncclUniqueId uid;
    std::memcpy(uid.internal, id.data(), NCCL_UNIQUE_ID_BYTES);
    check(a.init_rank(&comm_, world, uid, rank), "ncclCommInitRank");
  }
  ~RcclTransport() override {
    if (comm_ && !aborted_.load()) {
      try {
        api().destroy(comm_);
      } catch (...) {
      }
    }
  }
  void all_reduce(void* buf, size_t count, int dtype, hipStream_t s) override {
    if (aborted_.load()) throw std::runtime_error("all_reduce on an aborted communicator");
    check(api().all_reduce(buf, buf, count, static_cast<ncclDataType_t>(dtype), ncclSum, comm_, s),
          "ncclAllReduce");
  }
  void broadcast(void* buf, size_t count, int dtype, int root, hipStream_t s) override {
    if (aborted_.load()) throw std::runtime_error("broadcast on an aborted communicator");
    check(api().broadcast(buf, buf, count, static_cast<ncclDataType_t>(dtype), root, comm_, s),
          "ncclBroadcast");
  }
  int async_error() override {
    if (aborted_.load()) return -1;
    ncclResult_t r = ncclSuccess;
    check(api().async_error(comm_, &r), "ncclCommGetAsyncError");
    return static_cast<int>(r);
  }
  void abort() override {
    bool expect = false;
    if (comm_ && aborted_.compare_exchange_strong(expect, true)) api().abort(comm_);
  }
  const char* kind() const override { return "rccl"; }
  std::string library() const override { return api().path; }

 private:
  ncclComm_t comm_ = nullptr;
  std::atomic<bool> aborted_{false};
};

class LoopbackTransport final : public Transport {
 public:
  explicit LoopbackTransport(float f) : factor_(f) {}
  void all_reduce(void* buf, size_t count, int dtype, hipStream_t s) override {
    if (aborted_.load()) throw std::runtime_error("all_reduce on an aborted communicator");
    if (dtype != COMM_F32 && dtype != COMM_BF16)
      throw std::invalid_argument("loopback all_reduce: fp32 or bf16 only");
    comm_scale_inplace(buf, count, dtype, factor_, s);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
      throw std::runtime_error(std::string("loopback all_reduce: ") + hipGetErrorString(e));
  }
  void broadcast(void*, size_t, int, int root, hipStream_t) override {
    if (root != 0) throw std::invalid_argument("loopback broadcast: one rank, root 0");
  }
  int async_error() override { return aborted_.load() ? -1 : 0; }
  void abort() override { aborted_.store(true); }
  const char* kind() const override { return "loopback"; }

 private:
  float factor_;
  std::atomic<bool> aborted_{false};
};

}  // namespace

Comm::Comm(const std::string& id, int world, int rank, int device) : world_(world), rank_(rank) {
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("Comm: bad rank/world");
  t_.reset(new RcclTransport(id, world, rank, device));
}

Comm::Comm(std::unique_ptr<Transport> t, int world, int rank)
    : t_(std::move(t)), world_(world), rank_(rank) {}

Comm::~Comm() = default;

std::unique_ptr<Comm> Comm::shm(const std::string& name, int world, int rank, int device,
                                size_t slot_bytes, double timeout_s, double init_timeout_s) {
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("Comm: bad rank/world");
  return std::unique_ptr<Comm>(new Comm(
      make_shm_transport(name, world, rank, device, slot_bytes, timeout_s, init_timeout_s), world,
      rank));
}

std::unique_ptr<Comm> Comm::loopback(float factor) {
  return std::unique_ptr<Comm>(new Comm(std::unique_ptr<Transport>(new LoopbackTransport(factor)),
                                        1, 0));
}

void Comm::all_reduce(void* buf, size_t count, int dtype, hipStream_t s) {
  t_->all_reduce(buf, count, dtype, s);
}
void Comm::broadcast(void* buf, size_t count, int dtype, int root, hipStream_t s) {
  if (root < 0 || root >= world_) throw std::invalid_argument("broadcast: bad root");
  t_->broadcast(buf, count, dtype, root, s);
}
void Comm::host_all_reduce(void* buf, size_t count, int dtype) {
  shm_host_all_reduce(t_.get(), buf, count, dtype);
}
void Comm::host_broadcast(void* buf, size_t count, int dtype, int root) {
  if (root < 0 || root >= world_) throw std::invalid_argument("broadcast: bad root");
  shm_host_broadcast(t_.get(), buf, count, dtype, root);
}
int Comm::async_error() { return t_->async_error(); }
void Comm::abort() { t_->abort(); }

std::string Comm::unique_id() {
  ncclUniqueId uid;
  check(api().get_unique_id(&uid), "ncclGetUniqueId");
  return std::string(uid.internal, NCCL_UNIQUE_ID_BYTES);
}

std::string Comm::library() { return api().path; }

int Comm::rccl_version() {
  try {
    const RcclApi& a = api();
    int v = 0;
    if (a.get_version && a.get_version(&v) == ncclSuccess) return v;
  } catch (...) {
  }
  return -1;
}

bool Comm::rccl_available() {
  try {
    api();
    return true;
  } catch (...) {
    return false;
  }
}

}  // namespace dtr
