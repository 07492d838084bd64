// RCCL communicator owned by the native layer (SURVEY §2.3 "MI355X-native
// equivalent"): the gradient all-reduces of a training step are ops of the
// static Plan, issued on a dedicated comm HIP stream and ordered against the
// compute streams with hipEvents, instead of host-side c10d calls between plan
// segments.  Replaces Horovod's NCCL all-reduce of every gradient
// (/root/reference/resnet_model.py:115-117) and BroadcastGlobalVariablesHook
// (/root/reference/resnet_cifar_main.py:333).
//
// No second RCCL copy is loaded: the entry points are resolved from the
// librccl that PyTorch-ROCm already mapped into the process (dlopen with
// RTLD_NOLOAD), and the communicator is a fresh ncclCommInitRank over a
// ncclUniqueId the Python side distributes through the c10d TCP store.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>

namespace dtr {

// dtype codes (the RCCL ncclDataType_t values)
enum CommDtype : int { COMM_F32 = 7, COMM_BF16 = 9, COMM_F64 = 8, COMM_I64 = 4 };

struct CommImpl;

class Comm {
 public:
  // Collective: every rank of the job constructs one with the same id.
  Comm(const std::string& unique_id, int world, int rank, int device);
  ~Comm();
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;

  // SUM all-reduce, in place.  Stream-ordered; never blocks the host.
  void all_reduce(void* buf, size_t count, int dtype, hipStream_t s) const;
  void broadcast(void* buf, size_t count, int dtype, int root, hipStream_t s) const;
  // ncclCommGetAsyncError: 0 = ok, else the ncclResult_t (a peer died, a timeout...)
  int async_error() const;
  // ncclCommAbort: unblocks every pending collective of this rank (watchdog path)
  void abort();
  int world() const { return world_; }
  int rank() const { return rank_; }

  static std::string unique_id();   // ncclGetUniqueId, 128 opaque bytes
  static std::string library();     // path of the librccl the symbols come from

 private:
  std::unique_ptr<CommImpl> impl_;
  int world_, rank_;
};

}  // namespace dtr
