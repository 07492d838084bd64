// Communicator owned by the native layer (SURVEY §2.3 "MI355X-native
// equivalent"): the gradient all-reduces of a training step are ops of the
// static Plan, issued on a dedicated comm HIP stream and ordered against the
// compute streams with hipEvents, instead of host-side c10d calls between plan
// segments.  Replaces Horovod's NCCL all-reduce of every gradient
// (/root/reference/resnet_model.py:115-117) and BroadcastGlobalVariablesHook
// (/root/reference/resnet_cifar_main.py:333).
//
// One Comm interface, three transports behind it:
//   rccl      production: RCCL over xGMI.  No second RCCL copy is loaded: the
//             entry points are resolved from the librccl that PyTorch-ROCm
//             already mapped (dlopen RTLD_NOLOAD); a fresh ncclCommInitRank over
//             a ncclUniqueId the Python side distributes through the c10d store.
//   shm       rehearsal: host-staged all-reduce through a POSIX shared-memory
//             segment (comm_shm.cpp).  RCCL refuses two ranks on one device, so
//             this is how several ranks folded onto the one-GPU box run exactly
//             the plan ops, comm-stream events, issue threads and bf16 casts that
//             RCCL runs on 8 GPUs.  Deterministic rank-order sums, dead-peer and
//             timeout detection (async_error), abort that releases every peer.
//   loopback  diagnostics: a one-rank "all-reduce" that scales the buffer in
//             place by `factor` on the stream.  With factor 2 a bucket reduced
//             before its last gradient writer finished (or a writer landing on an
//             already-reduced range) shows up as a value that is not exactly 2x.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>

namespace dtr {

// dtype codes (the RCCL ncclDataType_t values)
enum CommDtype : int { COMM_F32 = 7, COMM_BF16 = 9, COMM_F64 = 8, COMM_I64 = 4 };
// async_error() codes (ncclResult_t values)
enum CommError : int { COMM_OK = 0, COMM_SYSTEM_ERROR = 2, COMM_INVALID_USAGE = 5,
                       COMM_REMOTE_ERROR = 6 };

size_t comm_dtype_bytes(int dtype);   // throws on an unknown code

class Transport {
 public:
  virtual ~Transport() = default;
  // SUM all-reduce, in place, ordered on stream s
  virtual void all_reduce(void* buf, size_t count, int dtype, hipStream_t s) = 0;
  virtual void broadcast(void* buf, size_t count, int dtype, int root, hipStream_t s) = 0;
  virtual int async_error() = 0;   // 0 ok, else a CommError / ncclResult_t
  virtual void abort() = 0;        // unblocks every pending collective of this rank
  virtual const char* kind() const = 0;
  virtual std::string library() const { return std::string(); }
};

class Comm {
 public:
  // RCCL: collective, every rank of the job constructs one with the same id.
  Comm(const std::string& unique_id, int world, int rank, int device);
  Comm(std::unique_ptr<Transport> t, int world, int rank);
  ~Comm();
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;

  // Collective (every rank, same name): the shared-memory rehearsal transport.
  // device < 0: host buffers only (host_all_reduce; CPU tests).
  // timeout_s bounds every collective's waits; init_timeout_s (<= 0: timeout_s) the
  // attach, i.e. the ranks' start-up skew.
  static std::unique_ptr<Comm> shm(const std::string& name, int world, int rank, int device,
                                   size_t slot_bytes, double timeout_s, double init_timeout_s);
  static std::unique_ptr<Comm> loopback(float factor);

  void all_reduce(void* buf, size_t count, int dtype, hipStream_t s);
  void broadcast(void* buf, size_t count, int dtype, int root, hipStream_t s);
  // shm transport only: the same collective on host memory (no HIP calls)
  void host_all_reduce(void* buf, size_t count, int dtype);
  void host_broadcast(void* buf, size_t count, int dtype, int root);
  int async_error();
  void abort();
  int world() const { return world_; }
  int rank() const { return rank_; }
  const char* transport() const { return t_->kind(); }
  std::string library_path() const { return t_->library(); }

  static std::string unique_id();   // ncclGetUniqueId, 128 opaque bytes
  static std::string library();     // path of the librccl the symbols come from
  static bool rccl_available();     // every RCCL entry point resolves (no throw)
  static int rccl_version();        // ncclGetVersion of the loaded librccl, -1 if unknown

 private:
  std::unique_ptr<Transport> t_;
  int world_, rank_;
};

// shm transport factory (comm_shm.cpp)
std::unique_ptr<Transport> make_shm_transport(const std::string& name, int world, int rank,
                                              int device, size_t slot_bytes, double timeout_s,
                                              double init_timeout_s);
// host entry points of the shm transport (throw if `t` is not one)
void shm_host_all_reduce(Transport* t, void* buf, size_t count, int dtype);
void shm_host_broadcast(Transport* t, void* buf, size_t count, int dtype, int root);

// loopback transport kernel (diag.hip): buf[i] *= factor, fp32 or bf16
void comm_scale_inplace(void* buf, size_t count, int dtype, float factor, hipStream_t s);

}  // namespace dtr
