// Shared-memory rehearsal transport of the native communicator (comm.h).
//
// Purpose: RCCL refuses two ranks on one device, so on a one-GPU box the
// world > 1 path of the training plan (bucket all-reduces as plan ops on the
// comm stream, the per-stream issue threads, the event fork/join, the bf16
// casts, broadcast-on-init) could never run.  This transport puts the same
// collectives behind the same Comm interface, host-staged:
//
//   D2H of this rank's chunk into its slot of a POSIX shm segment (stream-
//   ordered, then the issuing thread waits for the stream) -> barrier -> every
//   rank sums the slots in RANK ORDER (so all ranks compute the same bits, and a
//   test can predict them) -> barrier -> H2D of the sum.
//
// It blocks the issuing host thread -- the comm stream's issue thread in a
// threaded Plan::run, which is exactly where RCCL's enqueue happens -- while the
// main/side issue threads keep going.  Buckets larger than a slot go in chunks.
//
// Failure detection (the reference relies on MonitoredTrainingSession recovery,
// /root/reference/resnet_imagenet_main.py:363): every wait checks an abort flag
// in the segment, a deadline (timeout_s) and, every few ms, whether the peers it
// is waiting for still exist.  On failure it records COMM_REMOTE_ERROR (what
// ncclCommGetAsyncError reports for a dead peer), raises the segment's abort flag
// so every other rank fails fast too, and throws (the plan op fails, Plan::run
// raises in Python).
//
// Lifecycle: rank 0 creates the segment (O_EXCL, a name unique per job that the
// Python side distributes through the c10d store); the others open it; once all
// ranks have attached (first barrier) rank 0 unlinks the name, so a killed job
// leaves nothing behind in /dev/shm.
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "comm.h"

namespace dtr {

namespace {

constexpr uint64_t kMagic = 0x4454525348434f4dull;   // "DTRSHCOM"
constexpr int kMaxRanks = 64;

struct alignas(64) Line {
  std::atomic<uint64_t> v;
  char pad[64 - sizeof(std::atomic<uint64_t>)];
};

struct Header {
  std::atomic<uint64_t> magic;
  int32_t world;
  int32_t pad0;
  uint64_t slot_bytes;
  Line abort_flag;           // nonzero: some rank failed or aborted (its rank + 1)
  Line arrive[kMaxRanks];    // barrier generation reached by each rank
  Line pid[kMaxRanks];       // each rank's pid (dead-peer detection)
};

static_assert(std::atomic<uint64_t>::is_always_lock_free, "cross-process atomics");

size_t data_offset() { return (sizeof(Header) + 4095) & ~size_t(4095); }

using Clock = std::chrono::steady_clock;

inline uint16_t f2bf_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);   // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
inline float bf2f_bits(uint16_t b) {
  const uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

bool pid_alive(pid_t p) {
  if (p <= 0) return true;   // not attached yet: the deadline covers it
  if (::kill(p, 0) != 0 && errno == ESRCH) return false;
  // a zombie (exited, not yet reaped by its parent) still answers kill(0)
  char path[64];
  std::snprintf(path, sizeof(path), "/proc/%d/stat", (int)p);
  FILE* f = std::fopen(path, "r");
  if (!f) return true;
  char buf[512];
  const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[n] = 0;
  const char* rp = std::strrchr(buf, ')');
  if (rp && rp[1] == ' ' && (rp[2] == 'Z' || rp[2] == 'X')) return false;
  return true;
}

class ShmTransport final : public Transport {
 public:
  ShmTransport(const std::string& name, int world, int rank, int device, size_t slot_bytes,
               double timeout_s, double init_timeout_s)
      : name_(name), world_(world), rank_(rank), device_(device),
        slot_bytes_((slot_bytes + 63) & ~size_t(63)), timeout_s_(init_timeout_s) {
    if (world < 1 || world > kMaxRanks) throw std::invalid_argument("shm comm: world out of range");
    if (slot_bytes_ < 4096) throw std::invalid_argument("shm comm: slot_bytes < 4096");
    if (name.empty() || name[0] != '/' || name.find('/', 1) != std::string::npos)
      throw std::invalid_argument("shm comm: name must look like /dtr-...");
    size_ = data_offset() + (size_t)world * slot_bytes_;
    const auto deadline = Clock::now() + std::chrono::duration<double>(timeout_s_);
    int fd = -1;
    if (rank == 0) {
      fd = ::shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm comm: shm_open(create " + name + "): " + std::strerror(errno));
      owner_ = true;
      if (::ftruncate(fd, (off_t)size_) != 0) {
        const int e = errno;
        ::close(fd);
        ::shm_unlink(name.c_str());
        throw std::runtime_error(std::string("shm comm: ftruncate: ") + std::strerror(e));
      }
    } else {
      for (;;) {
        fd = ::shm_open(name.c_str(), O_RDWR, 0600);
        if (fd >= 0) {
          struct stat st;
          if (::fstat(fd, &st) == 0 && (size_t)st.st_size == size_) break;
          ::close(fd);
          fd = -1;
        }
        if (Clock::now() > deadline) throw std::runtime_error("shm comm: timed out opening " + name);
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
      }
    }
    void* p = ::mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (p == MAP_FAILED) {
      if (owner_) ::shm_unlink(name.c_str());
      throw std::runtime_error(std::string("shm comm: mmap: ") + std::strerror(errno));
    }
    base_ = static_cast<char*>(p);
    hdr_ = reinterpret_cast<Header*>(base_);
    if (rank == 0) {
      hdr_->world = world;
      hdr_->slot_bytes = slot_bytes_;
      hdr_->magic.store(kMagic, std::memory_order_release);
    } else {
      while (hdr_->magic.load(std::memory_order_acquire) != kMagic) {
        if (Clock::now() > deadline) {
          ::munmap(base_, size_);
          throw std::runtime_error("shm comm: segment never initialised by rank 0");
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
      if (hdr_->world != world || hdr_->slot_bytes != slot_bytes_) {
        ::munmap(base_, size_);
        throw std::runtime_error("shm comm: world / slot size differ between ranks");
      }
    }
    hdr_->pid[rank].v.store((uint64_t)::getpid(), std::memory_order_release);
    // pinned result staging (H2D source); pageable when there is no device
    if (device_ >= 0) {
      if (hipSetDevice(device_) != hipSuccess ||
          hipHostMalloc(&res_, slot_bytes_, hipHostMallocDefault) != hipSuccess) {
        res_ = nullptr;
        (void)hipGetLastError();
      } else {
        pinned_ = true;
      }
    }
    if (!res_) {
      host_res_.resize(slot_bytes_ / 8 + 1);
      res_ = host_res_.data();
    }
    try {
      barrier("attach");   // (the ranks' process start-up skew: the init timeout)
    } catch (...) {        // no destructor runs for a throwing constructor
      release();
      throw;
    }
    timeout_s_ = timeout_s;
    if (owner_) {
      ::shm_unlink(name_.c_str());
      unlinked_ = true;
    }
  }

  ~ShmTransport() override { release(); }

  void release() {
    if (pinned_) (void)hipHostFree(res_);
    pinned_ = false;
    res_ = nullptr;
    if (base_) ::munmap(base_, size_);
    base_ = nullptr;
    hdr_ = nullptr;
    if (owner_ && !unlinked_) ::shm_unlink(name_.c_str());
    unlinked_ = true;
  }

  void all_reduce(void* buf, size_t count, int dtype, hipStream_t s) override {
    check_stream(s);
    run_all_reduce(count, dtype, [&](char* slot, size_t off, size_t bytes) {
      dcheck(hipMemcpyAsync(slot, static_cast<char*>(buf) + off, bytes, hipMemcpyDeviceToHost, s),
             "D2H");
      dcheck(hipStreamSynchronize(s), "stream sync");
    }, [&](const char* res, size_t off, size_t bytes) {
      dcheck(hipMemcpyAsync(static_cast<char*>(buf) + off, res, bytes, hipMemcpyHostToDevice, s),
             "H2D");
      dcheck(hipStreamSynchronize(s), "stream sync");   // res_ is reused by the next chunk
    });
  }

  void broadcast(void* buf, size_t count, int dtype, int root, hipStream_t s) override {
    check_stream(s);
    run_broadcast(count, dtype, root, [&](char* slot, size_t off, size_t bytes) {
      dcheck(hipMemcpyAsync(slot, static_cast<char*>(buf) + off, bytes, hipMemcpyDeviceToHost, s),
             "D2H");
      dcheck(hipStreamSynchronize(s), "stream sync");
    }, [&](const char* res, size_t off, size_t bytes) {
      dcheck(hipMemcpyAsync(static_cast<char*>(buf) + off, res, bytes, hipMemcpyHostToDevice, s),
             "H2D");
      dcheck(hipStreamSynchronize(s), "stream sync");
    });
  }

  void host_all_reduce(void* buf, size_t count, int dtype) {
    char* b = static_cast<char*>(buf);
    run_all_reduce(count, dtype,
                   [&](char* slot, size_t off, size_t bytes) { std::memcpy(slot, b + off, bytes); },
                   [&](const char* res, size_t off, size_t bytes) { std::memcpy(b + off, res, bytes); });
  }

  void host_broadcast(void* buf, size_t count, int dtype, int root) {
    char* b = static_cast<char*>(buf);
    run_broadcast(count, dtype, root,
                  [&](char* slot, size_t off, size_t bytes) { std::memcpy(slot, b + off, bytes); },
                  [&](const char* res, size_t off, size_t bytes) { std::memcpy(b + off, res, bytes); });
  }

  int async_error() override { return err_.load(); }

  void abort() override {
    aborted_.store(true);
    uint64_t z = 0;
    hdr_->abort_flag.v.compare_exchange_strong(z, (uint64_t)rank_ + 1);
    int ok = COMM_OK;
    err_.compare_exchange_strong(ok, COMM_REMOTE_ERROR);
  }

  const char* kind() const override { return "shm"; }
  std::string library() const override { return "shm:" + name_; }

 private:
  char* slot(int r) const { return base_ + data_offset() + (size_t)r * slot_bytes_; }

  [[noreturn]] void fail(const std::string& why) {
    int ok = COMM_OK;
    err_.compare_exchange_strong(ok, COMM_REMOTE_ERROR);
    uint64_t z = 0;
    hdr_->abort_flag.v.compare_exchange_strong(z, (uint64_t)rank_ + 1);
    throw std::runtime_error("shm comm (rank " + std::to_string(rank_) + "): " + why);
  }

  void dcheck(hipError_t e, const char* what) {
    if (e != hipSuccess) fail(std::string(what) + ": " + hipGetErrorString(e));
  }

  void check_stream(hipStream_t s) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone)
      throw std::runtime_error("shm comm: host-staged collectives cannot be captured in a hipGraph");
  }

  void entry_checks() {
    if (aborted_.load()) throw std::runtime_error("collective on an aborted communicator");
    if (err_.load() != COMM_OK) throw std::runtime_error("collective on a failed communicator");
    const uint64_t a = hdr_->abort_flag.v.load(std::memory_order_acquire);
    if (a) fail("the job was aborted by rank " + std::to_string((long long)a - 1));
  }

  void barrier(const char* what) {
    const uint64_t g = ++gen_;
    hdr_->arrive[rank_].v.store(g, std::memory_order_release);
    const auto t0 = Clock::now();
    const auto deadline = t0 + std::chrono::duration<double>(timeout_s_);
    auto next_probe = t0 + std::chrono::milliseconds(5);
    for (int q = 0; q < world_; ++q) {
      unsigned spins = 0;
      while (hdr_->arrive[q].v.load(std::memory_order_acquire) < g) {
        const uint64_t a = hdr_->abort_flag.v.load(std::memory_order_relaxed);
        if (a) fail(std::string(what) + ": the job was aborted by rank " +
                    std::to_string((long long)a - 1));
        if (aborted_.load(std::memory_order_relaxed)) fail(std::string(what) + ": aborted");
        if (++spins < 256) continue;
        if (spins < 4096) {
          std::this_thread::yield();
          continue;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
        const auto now = Clock::now();
        if (now >= next_probe) {
          next_probe = now + std::chrono::milliseconds(5);
          const pid_t p = (pid_t)hdr_->pid[q].v.load(std::memory_order_acquire);
          if (!pid_alive(p))
            fail(std::string(what) + ": rank " + std::to_string(q) + " (pid " + std::to_string(p) +
                 ") is gone");
          if (now > deadline)
            fail(std::string(what) + ": timed out after " + std::to_string(timeout_s_) +
                 " s waiting for rank " + std::to_string(q));
        }
      }
    }
  }

  template <class In, class Out>
  void run_all_reduce(size_t count, int dtype, In copy_in, Out copy_out) {
    entry_checks();
    const size_t esz = comm_dtype_bytes(dtype);
    if (dtype == COMM_I64) throw std::invalid_argument("shm all_reduce: fp32 / bf16 / fp64 only");
    const size_t per = slot_bytes_ / esz;
    for (size_t e0 = 0; e0 < count; e0 += per) {
      const size_t n = std::min(per, count - e0);
      copy_in(slot(rank_), e0 * esz, n * esz);
      barrier("all_reduce");
      reduce(n, dtype);
      barrier("all_reduce");   // every rank has read every slot: they may be refilled
      copy_out(static_cast<const char*>(res_), e0 * esz, n * esz);
    }
  }

  template <class In, class Out>
  void run_broadcast(size_t count, int dtype, int root, In copy_in, Out copy_out) {
    entry_checks();
    const size_t esz = comm_dtype_bytes(dtype);
    const size_t per = slot_bytes_ / esz;
    for (size_t e0 = 0; e0 < count; e0 += per) {
      const size_t n = std::min(per, count - e0);
      if (rank_ == root) copy_in(slot(root), e0 * esz, n * esz);
      barrier("broadcast");
      if (rank_ != root) std::memcpy(res_, slot(root), n * esz);
      barrier("broadcast");
      if (rank_ != root) copy_out(static_cast<const char*>(res_), e0 * esz, n * esz);
    }
  }

  // res_[i] = slot(0)[i] + slot(1)[i] + ... in rank order (identical bits on every rank)
  void reduce(size_t n, int dtype) {
    if (dtype == COMM_F32) {
      float* r = static_cast<float*>(res_);
      std::memcpy(r, slot(0), n * 4);
      for (int q = 1; q < world_; ++q) {
        const float* s = reinterpret_cast<const float*>(slot(q));
        for (size_t i = 0; i < n; ++i) r[i] += s[i];
      }
    } else if (dtype == COMM_F64) {
      double* r = static_cast<double*>(res_);
      std::memcpy(r, slot(0), n * 8);
      for (int q = 1; q < world_; ++q) {
        const double* s = reinterpret_cast<const double*>(slot(q));
        for (size_t i = 0; i < n; ++i) r[i] += s[i];
      }
    } else {   // bf16: fp32 sum in rank order, one RNE rounding
      uint16_t* r = static_cast<uint16_t*>(res_);
      for (size_t i = 0; i < n; ++i) {
        float acc = bf2f_bits(reinterpret_cast<const uint16_t*>(slot(0))[i]);
        for (int q = 1; q < world_; ++q) acc += bf2f_bits(reinterpret_cast<const uint16_t*>(slot(q))[i]);
        r[i] = f2bf_rne(acc);
      }
    }
  }

  std::string name_;
  int world_, rank_, device_;
  size_t slot_bytes_, size_ = 0;
  double timeout_s_;
  char* base_ = nullptr;
  Header* hdr_ = nullptr;
  bool owner_ = false, unlinked_ = false, pinned_ = false;
  void* res_ = nullptr;
  std::vector<uint64_t> host_res_;
  uint64_t gen_ = 0;
  std::atomic<int> err_{COMM_OK};
  std::atomic<bool> aborted_{false};
};

ShmTransport* as_shm(Transport* t) {
  auto* s = dynamic_cast<ShmTransport*>(t);
  if (!s) throw std::invalid_argument("host collectives need the shm transport");
  return s;
}

}  // namespace

std::unique_ptr<Transport> make_shm_transport(const std::string& name, int world, int rank,
                                              int device, size_t slot_bytes, double timeout_s,
                                              double init_timeout_s) {
  return std::unique_ptr<Transport>(new ShmTransport(name, world, rank, device, slot_bytes,
                                                     timeout_s,
                                                     init_timeout_s > 0 ? init_timeout_s : timeout_s));
}

void shm_host_all_reduce(Transport* t, void* buf, size_t count, int dtype) {
  as_shm(t)->host_all_reduce(buf, count, dtype);
}

void shm_host_broadcast(Transport* t, void* buf, size_t count, int dtype, int root) {
  as_shm(t)->host_broadcast(buf, count, dtype, root);
}

}  // namespace dtr
