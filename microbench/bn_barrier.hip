// BatchNorm grid-barrier microbenchmark (MI355X): the persistent CIFAR step's per-BN
// round trip (csrc/cifar_persist.hip bn_sums / grid_arrive / grid_wait / acc_read) in
// isolation, to choose its arrival / poll scheme by measurement.
//
// One 512-thread workgroup per CU (as the persistent kernels), G = 64 / 128 / 256.  Per
// barrier every workgroup:
//   work   ~W ns of VALU (a stand-in for the conv between two BatchNorms; W = 0 or 1000)
//   sums   threads c < 64 add two fp64 values into replica (block % REP) of acc[REP][2][64]
//          (memory-side atomics, no return), then every wave drains (vmcnt(0)) + barrier
//   arrive lane 0 adds 1 to the arrival counter (scheme below)
//   wait   poll until every workgroup of this barrier has arrived (bounded: 2 s)
//   read   threads c < 64 read the 2 x REP replica values of their channel (sc1 loads)
// Arrival / poll schemes:
//   flat    one counter line; lane 0 of wave 0 polls it (s_sleep 1 between polls) --
//           the round-4 kernels
//   shard8  8 counters on 8 lines, workgroup b adds to b % 8 (one XCD each under
//           round-robin placement); lanes 0-7 of wave 0 poll all 8 with ONE load
//           instruction, done when every shard holds its count
//   flat4w  one counter, lane 0 of waves 0-3 poll it independently (staggered start),
//           the first to see it complete sets an LDS flag the others read
//   shard4w shard8's counters polled by waves 0-3 (each wave one 8-lane load)
// Time per barrier = (kernel with B barriers - kernel with the work alone) / B, median of
// 5.  Prints a markdown table (profiles/bn_barrier.md).
//
//   hipcc --offload-arch=gfx950 -O3 -o microbench/bn_barrier microbench/bn_barrier.hip
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

constexpr long long kSpinTicks = 200000000;   // 2 s at 100 MHz
constexpr int C = 64;

enum Mode { FLAT = 0, SHARD8 = 1, FLAT4W = 2, SHARD4W = 3, SHARD8P2 = 4, SHARD8P4 = 5, SHARD8S4 = 6, SHARD8S16 = 7, SHARD16 = 8, NMODES = 9 };
static const char* kNames[NMODES] = {"flat", "shard8", "flat4w", "shard4w", "shard8 2-in-flight", "shard8 4-in-flight", "shard8 sleep 4", "shard8 sleep 16", "shard16"};

struct Ctl {
  unsigned cnt[16][32];   // 16 counter lines (flat uses line 0; shards lines 0-7)
  unsigned fail;
  unsigned pad[31];
  double acc[16][2][C];   // [REP][2][C]
  double sink[1024];
};

__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_agent_d(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int MODE, int REP>
__global__ void __launch_bounds__(512, 1) bn_barrier_kernel(Ctl* c, int iters, int work, int do_sums) {
  __shared__ int flag[4];
  __shared__ double tbl[2 * C];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int G = gridDim.x;
  const int shard = blockIdx.x % (MODE == SHARD16 ? 16 : 8);
  // per-shard arrival counts (shard s: blocks b with b % 8 == s)
  float x = (float)tid;
  bool ok = true;
  for (int it = 1; it <= iters && ok; ++it) {
    // ---- work ----
    for (int i = 0; i < work; ++i) x = x * 1.0001f + 0.5f;
    if (do_sums < 0) continue;   // the work alone (the baseline subtracted)
    // ---- sums ----
    if (do_sums && tid < C) {
      double* p = &c->acc[blockIdx.x % REP][0][tid];
      __builtin_amdgcn_global_atomic_fadd_f64((__attribute__((address_space(1))) double*)p, (double)x);
      __builtin_amdgcn_global_atomic_fadd_f64((__attribute__((address_space(1))) double*)(p + C),
                                              (double)x * x);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid < 4) flag[tid] = 0;
    __syncthreads();
    // ---- arrive ----
    if (tid == 0) {
      unsigned* ctr = (MODE == FLAT || MODE == FLAT4W) ? &c->cnt[0][0] : &c->cnt[shard][0];
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // ---- wait ----
    const int pollers = (MODE == FLAT4W || MODE == SHARD4W) ? 4 : 1;
    if (MODE == SHARD8P2 || MODE == SHARD8P4) {
      // one wave, lanes 0-7, NP polls in flight: each check waits for the oldest load only
      constexpr int NP = MODE == SHARD8P2 ? 2 : 4;
      if (tid < 8) {
        const unsigned target = (unsigned)it * (unsigned)((G - tid + 7) / 8);
        const unsigned* ctr = &c->cnt[tid][0];
        const long long t0 = wall_clock64();
        unsigned v[NP];
#pragma unroll
        for (int j = 0; j < NP; ++j) {
          v[j] = ld_agent(ctr);
          if (j + 1 < NP) __builtin_amdgcn_s_sleep(2);
        }
        bool fin = false;
        while (!fin) {
#pragma unroll
          for (int j = 0; j < NP; ++j) {
            const bool done = v[j] >= target;
            if (__builtin_amdgcn_ballot_w64(!done) == 0) {
              fin = true;
              break;
            }
            v[j] = ld_agent(ctr);   // re-issue in this slot (the others are still in flight)
            __builtin_amdgcn_s_sleep(2);
          }
          if (!fin && wall_clock64() - t0 > kSpinTicks) {
            if (tid == 0) flag[1] = 1;
            break;
          }
        }
      }
    } else if (wave < pollers) {
      const bool sh = MODE != FLAT && MODE != FLAT4W;
      const int lanes = MODE == SHARD16 ? 16 : sh ? 8 : 1;
      if (lane < lanes) {
        const unsigned per = MODE == SHARD16 ? (unsigned)((G - lane + 15) / 16)
                             : sh ? (unsigned)((G - lane + 7) / 8) : (unsigned)G;
        const unsigned target = per * (unsigned)it;
        const unsigned* ctr = &c->cnt[sh ? lane : 0][0];
        const long long t0 = wall_clock64();
        for (int i = 0; i < wave; ++i) __builtin_amdgcn_s_sleep(8);   // stagger the pollers
        for (;;) {
          const bool mine = ld_agent(ctr) >= target;
          // every polling lane of this wave complete? (exec = the polling lanes)
          const bool all = __builtin_amdgcn_read_exec() == __builtin_amdgcn_ballot_w64(mine);
          if (all) {
            if (lane == 0) __hip_atomic_store(&flag[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            break;
          }
          if (pollers > 1 &&
              __hip_atomic_load(&flag[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
            break;
          if (MODE == SHARD8S4) __builtin_amdgcn_s_sleep(4);
          else if (MODE == SHARD8S16) __builtin_amdgcn_s_sleep(16);
          else __builtin_amdgcn_s_sleep(1);
          if (wall_clock64() - t0 > kSpinTicks) {
            __hip_atomic_fetch_add(&c->fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (lane == 0) __hip_atomic_store(&flag[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            break;
          }
        }
      }
    }
    __syncthreads();
    ok = flag[1] == 0;
    // ---- read ----
    if (do_sums && tid < C) {
      double a[REP], b[REP];
#pragma unroll
      for (int r = 0; r < REP; ++r) {
        a[r] = ld_agent_d(&c->acc[r][0][tid]);
        b[r] = ld_agent_d(&c->acc[r][1][tid]);
      }
      double s1 = 0, s2 = 0;
#pragma unroll
      for (int r = 0; r < REP; ++r) {
        s1 += a[r];
        s2 += b[r];
      }
      tbl[tid] = s1;
      tbl[C + tid] = s2;
    }
    __syncthreads();
    x += (float)tbl[lane] * 1e-30f;
  }
  if (tid == 0 && x == 12345.f) c->sink[blockIdx.x] = x;
}

template <int MODE, int REP>
static float run(Ctl* c, int G, int iters, int work, int sums, unsigned* fail) {
  CK(hipMemset(c, 0, sizeof(Ctl)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  hipLaunchKernelGGL((bn_barrier_kernel<MODE, REP>), dim3(G), dim3(512), 0, 0, c, iters, work, sums);
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

template <int MODE, int REP>
static float per_barrier(Ctl* c, int G, int work, int sums, bool* bad) {
  const int B = 2000;
  std::vector<float> t;
  for (int r = 0; r < 5; ++r) {
    unsigned f = 0;
    const float t1 = run<MODE, REP>(c, G, B, work, sums, &f);
    if (f) *bad = true;
    // the work alone (same grid, no sums / barrier traffic)
    const float t0 = run<MODE, REP>(c, G, B, work, -1, &f);
    t.push_back((t1 - t0) * 1000.f / B);
  }
  return median(t);
}

int main() {
  Ctl* c;
  CK(hipMalloc(&c, sizeof(Ctl)));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  std::printf("# BatchNorm grid barrier schemes (%s, %d CUs)\n\n", prop.name, prop.multiProcessorCount);
  std::printf("us per barrier (sums + drain + arrive + wait + sums read; minus the same kernel on one "
              "kernel without the barrier traffic), median of 5 launches of 2000 barriers, 512-thread workgroups, one per CU. "
              "`microbench/bn_barrier.hip`.\n\n");
  std::printf("| workgroups | work (dependent FMAs) | REP |");
  for (int m = 0; m < NMODES; ++m) std::printf(" %s |", kNames[m]);
  std::printf("\n|---|---|---|");
  for (int m = 0; m < NMODES; ++m) std::printf("---|");
  std::printf("\n");
  for (int G : {64, 128, 256}) {
    for (int work : {0, 400}) {
      for (int rep : {4, 8}) {
        bool bad = false;
        float r[NMODES];
        if (rep != 4) continue;
        r[0] = per_barrier<FLAT, 4>(c, G, work, 1, &bad);
        r[1] = per_barrier<SHARD8, 4>(c, G, work, 1, &bad);
        r[2] = per_barrier<FLAT4W, 4>(c, G, work, 1, &bad);
        r[3] = per_barrier<SHARD4W, 4>(c, G, work, 1, &bad);
        r[4] = per_barrier<SHARD8P2, 4>(c, G, work, 1, &bad);
        r[5] = per_barrier<SHARD8P4, 4>(c, G, work, 1, &bad);
        r[6] = per_barrier<SHARD8S4, 4>(c, G, work, 1, &bad);
        r[7] = per_barrier<SHARD8S16, 4>(c, G, work, 1, &bad);
        r[8] = per_barrier<SHARD16, 4>(c, G, work, 1, &bad);
        std::printf("| %d | %d | %d |", G, work, rep);
        for (int m = 0; m < NMODES; ++m) std::printf(" %.2f |", r[m]);
        std::printf("%s\n", bad ? " FAIL (timed-out barrier)" : "");
        std::fflush(stdout);
      }
    }
  }
  CK(hipFree(c));
  return 0;
}
