// Grid-barrier microbenchmark (MI355X): what a persistent multi-layer kernel would
// pay per dependent layer, against the kernel boundary it would replace.
//
// For a persistent CIFAR stage kernel ("build, don't cite"), every conv
// -> BatchNorm -> conv dependency is a grid-wide sync.  Measured here, per sync, at
// 32 / 64 / 128 / 256 participating workgroups (256 threads, one per CU unless
// stated):
//   boundary   back-to-back dependent launches of an empty kernel (same stream)
//   flat       one monotonic agent-scope counter: lane 0 adds, then polls it with
//              relaxed agent-scope loads (L1 bypass) + s_sleep
//   flat+fence the same with the release fence before the add and the acquire fence
//              after the poll that a barrier publishing plain-stored data needs
//   xcd1       flat, all participants on ONE XCD (grid of 8 x N, only the blocks of
//              one blockIdx % 8 class take part: they share an XCD and its L2)
//   hier       XCD-hierarchical: per-XCD counter, the XCD's last arriver adds to a
//              top counter, everyone polls the top counter
// Time per sync = (kernel with B syncs - kernel with 0 syncs) / B, median of 5.
// Every spin is bounded (wall clock); a timed-out barrier reports FAIL, the kernel
// still drains.  The XCC id of every participant is read (HW_REG_XCC_ID) to verify
// the one-XCD placement.
//
//   hipcc --offload-arch=gfx950 -O3 -o microbench/grid_barrier microbench/grid_barrier.hip
//   microbench/grid_barrier > profiles/grid_barrier.md
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

constexpr long long kSpinTicks = 200000000;   // 2 s at 100 MHz: bound of every wait

enum Mode { FLAT = 0, FLAT_FENCE = 1, XCD1 = 2, HIER = 3 };

struct Ctl {
  unsigned top;         // flat / top-level counter
  unsigned pad0[31];
  unsigned xcd[8][32];  // per-XCD counters (own 128-B lines)
  unsigned fail;
};

__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int xcc_id() {
  // s_getreg_b32 hwreg(HW_REG_XCC_ID, 0, 4): id 20, offset 0, size 4
  return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 15;
}

__device__ bool wait_ge(const unsigned* p, unsigned target, Ctl* c) {
  const long long t0 = wall_clock64();
  while (ld_agent(p) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (wall_clock64() - t0 > kSpinTicks) {
      __hip_atomic_fetch_add(&c->fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  return true;
}

__global__ void __launch_bounds__(256) barrier_kernel(Ctl* c, int iters, int mode, int n_part,
                                                      int per_xcd, int* xcc_out) {
  int part = blockIdx.x;
  if (mode == XCD1) {
    if (blockIdx.x % 8 != 0) return;   // only one blockIdx % 8 class takes part
    part = blockIdx.x / 8;
  }
  if (threadIdx.x == 0 && xcc_out) xcc_out[part] = xcc_id();
  const int xcd = blockIdx.x % 8;      // shared-XCD class (hier)
  bool ok = true;
  for (int it = 1; it <= iters && ok; ++it) {
    __syncthreads();
    if (threadIdx.x == 0) {
      if (mode == FLAT_FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      if (mode == HIER) {
        const unsigned prev =
            __hip_atomic_fetch_add(&c->xcd[xcd][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev + 1 == (unsigned)(it * per_xcd))   // this XCD's last arriver
          __hip_atomic_fetch_add(&c->top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = wait_ge(&c->top, (unsigned)(it * 8), c);
      } else {
        __hip_atomic_fetch_add(&c->top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = wait_ge(&c->top, (unsigned)(it * n_part), c);
      }
      if (mode == FLAT_FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    ok = ld_agent(&c->fail) == 0;
  }
}

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1023) p[0] = 1;   // never true: keeps the launch non-trivial
}

static float time_barrier(Ctl* c, int iters, int mode, int n, int* xcc, unsigned* fail) {
  const int grid = mode == XCD1 ? 8 * n : n;
  CK(hipMemset(c, 0, sizeof(Ctl)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  hipLaunchKernelGGL(barrier_kernel, dim3(grid), dim3(256), 0, 0, c, iters, mode, n, n / 8, xcc);
  CK(hipGetLastError());
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipMemcpy(fail, &c->fail, 4, hipMemcpyDeviceToHost));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms;
}

static float median(std::vector<float> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  Ctl* c;
  int* xcc;
  CK(hipMalloc(&c, sizeof(Ctl)));
  CK(hipMalloc(&xcc, 4096 * sizeof(int)));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  std::printf("# Grid barrier vs kernel boundary (%s, %d CUs)\n\n", prop.name,
              prop.multiProcessorCount);
  std::printf("Per-sync cost in us (median of 5 launches; B = 2000 syncs per launch minus a "
              "0-sync launch). `microbench/grid_barrier.hip`.\n\n");
  std::printf("| workgroups | boundary | flat | flat+fence | xcd1 (one XCD) | hier (per-XCD) | "
              "xcd1 XCC ids |\n|---|---|---|---|---|---|---|\n");
  const int B = 2000;
  for (int n : {32, 64, 128, 256}) {
    // kernel boundary: B dependent launches of n workgroups
    std::vector<float> tb;
    for (int r = 0; r < 5; ++r) {
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      hipLaunchKernelGGL(empty_kernel, dim3(n), dim3(256), 0, 0, nullptr);
      CK(hipEventRecord(a, 0));
      for (int i = 0; i < B; ++i) hipLaunchKernelGGL(empty_kernel, dim3(n), dim3(256), 0, 0, nullptr);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      tb.push_back(ms * 1000.f / B);
      CK(hipEventDestroy(a));
      CK(hipEventDestroy(b));
    }
    float res[4];
    bool bad = false;
    for (int mode : {FLAT, FLAT_FENCE, XCD1, HIER}) {
      if (mode == HIER && n % 8) {
        res[mode] = -1;
        continue;
      }
      std::vector<float> t;
      for (int r = 0; r < 5; ++r) {
        unsigned f0 = 0, f1 = 0;
        const float t0 = time_barrier(c, 0, mode, n, nullptr, &f0);
        const float t1 = time_barrier(c, B, mode, n, mode == XCD1 ? xcc : nullptr, &f1);
        if (f1) bad = true;
        t.push_back((t1 - t0) * 1000.f / B);
      }
      res[mode] = median(t);
    }
    std::vector<int> ids(n);
    CK(hipMemcpy(ids.data(), xcc, n * sizeof(int), hipMemcpyDeviceToHost));
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    char idb[64] = {0};
    int o = 0;
    for (int v : ids) o += std::snprintf(idb + o, sizeof(idb) - o, "%s%d", o ? "," : "", v);
    std::printf("| %d | %.2f | %.2f | %.2f | %.2f | %.2f | %s |%s\n", n, median(tb), res[FLAT],
                res[FLAT_FENCE], res[XCD1], res[HIER], idb, bad ? " FAIL (timed-out barrier)" : "");
    std::fflush(stdout);
  }
  CK(hipFree(c));
  CK(hipFree(xcc));
  return 0;
}
