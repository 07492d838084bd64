// BatchNorm grid barrier: memory-side fp64 atomics + counter (the persistent CIFAR step's
// scheme since round 5: csrc/cifar_persist.hip bn_sums / grid_arrive / grid_wait / acc_read)
// against tagged slots, where the partial sums ARE the arrival:
//   atom   threads c < ch add (s1, s2) into fp64 replica blockIdx % 4 (no return), every
//          wave drains (vmcnt(0)), lane 0 adds 1 to its shard (8 lines), lanes 0-7 of wave 0
//          poll the shards, then threads c < ch read the 4 replicas of their channel
//   slot   thread c < ch writes ONE 16-byte entry {s1, s2, tag, tag ^ s1 ^ s2} (fp32 bits,
//          tag = barrier number) into its workgroup's row of buffer (k & 1) with a
//          write-through store: no drain, no counter.  Every thread then polls a fixed
//          share of the G x ch entries until all carry this barrier's tag and a matching
//          check word (a torn 16-byte write fails the check and is read again), sums its
//          share in a fixed order and the shares are folded through LDS -- the same total
//          on every workgroup, bitwise.  Two buffers: a workgroup writes barrier k + 2's
//          entry only after barrier k + 1, by which time every reader of k is done.
//   int    the sums as 64-bit fixed point (2^-15) shifted left 9 bits, plus 1: ONE memory-side
//          integer add per (channel, stat) carries the partial sum AND the arrival (low 9
//          bits count arrivals, exact and order-independent).  No drain, no counter: threads
//          c < ch poll their channel's 2 x 4 replica words until every count is complete;
//          the polled values are the sums
//   int1   as int, but lanes 0-3 poll channel 0's s1 words only, then every channel's words
//          are read (and re-read while any count is short)
// Every barrier uses its own accumulator lines (as every BN of the step does).
// us per barrier = (kernel with B barriers - the work alone) / B, median of 5.
//
//   hipcc --offload-arch=gfx950 -O3 -o microbench/bn_slots microbench/bn_slots.hip
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
constexpr int CMAX = 64, GMAX = 256, NT = 512;

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct Ctl {
  unsigned cnt[16][32];
  unsigned fail;
  unsigned bad;
  unsigned pad[30];
  u32x4 slot[2][GMAX][CMAX];
  double sink[1024];
};

__device__ __forceinline__ unsigned ld_agent(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_agent_d(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return reinterpret_cast<T*>(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ void st_wt_b128(u32x4* base, int idx, u32x4 v) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(base), 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, idx * 16, 0, 16);
}
__device__ __forceinline__ u32x4 ld_wt_b128(const u32x4* base, int idx) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(const_cast<u32x4*>(base)), 0,
                                                    0x7fffffff, 0x00020000);
  return __builtin_amdgcn_raw_buffer_load_b128(rs, idx * 16, 0, 16);
}

enum Mode { ATOM = 0, SLOT = 1, INT = 2, INT1 = 3, INT2 = 4 };
constexpr int NBAR = 2000;
struct Acc {   // per barrier: fp64 [4][2][CMAX] or fixed-point u64 [4][2][CMAX]
  union {
    double d[4][2][CMAX];
    unsigned long long q[4][2][CMAX];
    unsigned long long q2[4][4][CMAX];   // INT2: [rep][s1 hi, s1 lo, s2 hi, s2 lo][c]
  };
};
__device__ __forceinline__ unsigned long long ld_agent_q(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr int FRAC = 15, CBITS = 9;
__device__ __forceinline__ unsigned long long fx(float v) {
  return ((unsigned long long)llrint((double)v * (double)(1 << FRAC)) << CBITS) + 1ull;
}
__device__ __forceinline__ double unfx(unsigned long long w, unsigned n) {
  return (double)((long long)(w - n) >> CBITS) / (double)(1 << FRAC);
}
// INT2: v * 2^60 split into hi * 2^46 + lo (0 <= lo < 2^46), each word (part << 9) + 1
__device__ __forceinline__ void fx2(float v, unsigned long long& hi, unsigned long long& lo) {
  const double d = ldexp((double)v, 60);
  const double h = floor(ldexp(d, -46));
  const double l = rint(d - ldexp(h, 46));
  hi = ((unsigned long long)(long long)h << CBITS) + 1ull;
  lo = ((unsigned long long)(long long)l << CBITS) + 1ull;
}
__device__ __forceinline__ double unfx2(unsigned long long hi, unsigned long long lo, unsigned n) {
  return ldexp((double)((long long)(hi - n) >> CBITS), -14) +
         ldexp((double)((long long)(lo - n) >> CBITS), -60);
}

template <int MODE>
__global__ void __launch_bounds__(NT, 1) bar_kernel(Ctl* c, Acc* accs, int iters, int work, int do_sums, int ch) {
  __shared__ int flag[4];
  __shared__ double red[2][NT];
  __shared__ double tbl[2 * CMAX];
  const int tid = threadIdx.x;
  const int G = gridDim.x;
  float x = (float)(tid % 61) * 0.01f + 1.f;
  bool ok = true;
  if (tid < 4) flag[tid] = 0;
  __syncthreads();
  for (int it = 1; it <= iters && ok; ++it) {
    for (int i = 0; i < work; ++i) x = x * 1.0001f + 0.5f;
    if (do_sums < 0) continue;
    const float s1 = x + (float)blockIdx.x, s2 = x * x;
    Acc* A = accs + (it - 1);
    if (MODE == INT2) {
      if (tid < ch) {
        unsigned long long h1, l1, h2, l2;
        fx2(s1, h1, l1);
        fx2(s2, h2, l2);
        unsigned long long* p = &A->q2[blockIdx.x % 4][0][tid];
        __hip_atomic_fetch_add(p, h1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(p + CMAX, l1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(p + 2 * CMAX, h2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(p + 3 * CMAX, l2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const long long t0 = wall_clock64();
      int fail = 0;
      if (tid < 4) {
        const unsigned want = (unsigned)((G - tid + 3) / 4);
        for (;;) {
          const bool done = (unsigned)(ld_agent_q(&A->q2[tid][0][0]) & ((1u << CBITS) - 1)) == want;
          if (__builtin_amdgcn_ballot_w64(!done) == 0) break;
          __builtin_amdgcn_s_sleep(1);
          if (wall_clock64() - t0 > kSpinTicks) {
            fail = 1;
            break;
          }
        }
      }
      if (fail) flag[1] = 1;
      __syncthreads();
      if (tid < ch) {
        unsigned long long w[16];
        for (;;) {
          bool done = true;
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int j = 0; j < 4; ++j) w[4 * r + j] = ld_agent_q(&A->q2[r][j][tid]);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const unsigned want = (unsigned)((G - r + 3) / 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) done = done && (unsigned)(w[4 * r + j] & ((1u << CBITS) - 1)) == want;
          }
          if (done) break;
          __builtin_amdgcn_s_sleep(1);
          if (wall_clock64() - t0 > kSpinTicks) {
            fail = 1;
            break;
          }
        }
        unsigned long long h1 = 0, l1 = 0, h2 = 0, l2 = 0;
        unsigned n = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          h1 += w[4 * r];
          l1 += w[4 * r + 1];
          h2 += w[4 * r + 2];
          l2 += w[4 * r + 3];
          n += (unsigned)((G - r + 3) / 4);
        }
        tbl[tid] = unfx2(h1, l1, n);
        tbl[CMAX + tid] = unfx2(h2, l2, n);
        if (fail) flag[1] = 1;
      }
      __syncthreads();
      ok = flag[1] == 0;
    } else if (MODE == INT || MODE == INT1) {
      if (tid < ch) {
        unsigned long long* p = &A->q[blockIdx.x % 4][0][tid];
        __hip_atomic_fetch_add(p, fx(s1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(p + CMAX, fx(s2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const long long t0 = wall_clock64();
      int fail = 0;
      if (MODE == INT1 && tid < 4) {   // channel 0's s1 words of the 4 replicas
        const unsigned want = (unsigned)((G - tid + 3) / 4);
        for (;;) {
          const bool done = (unsigned)(ld_agent_q(&A->q[tid][0][0]) & ((1u << CBITS) - 1)) == want;
          if (__builtin_amdgcn_ballot_w64(!done) == 0) break;
          __builtin_amdgcn_s_sleep(1);
          if (wall_clock64() - t0 > kSpinTicks) {
            fail = 1;
            break;
          }
        }
      }
      if (MODE == INT1) {
        if (fail) flag[1] = 1;
        __syncthreads();
      }
      if (tid < ch) {
        unsigned long long w[8];
        for (;;) {
          bool done = true;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            w[2 * r] = ld_agent_q(&A->q[r][0][tid]);
            w[2 * r + 1] = ld_agent_q(&A->q[r][1][tid]);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const unsigned want = (unsigned)((G - r + 3) / 4);
            done = done && (unsigned)(w[2 * r] & ((1u << CBITS) - 1)) == want &&
                   (unsigned)(w[2 * r + 1] & ((1u << CBITS) - 1)) == want;
          }
          if (done) break;
          __builtin_amdgcn_s_sleep(1);
          if (wall_clock64() - t0 > kSpinTicks) {
            fail = 1;
            break;
          }
        }
        double a = 0.0, b = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const unsigned n = (unsigned)((G - r + 3) / 4);
          a += unfx(w[2 * r], n);
          b += unfx(w[2 * r + 1], n);
        }
        tbl[tid] = a;
        tbl[CMAX + tid] = b;
        if (fail) flag[1] = 1;
      }
      __syncthreads();
      ok = flag[1] == 0;
    } else if (MODE == ATOM) {
      if (tid < ch) {
        double* p = &A->d[blockIdx.x % 4][0][tid];
        __builtin_amdgcn_global_atomic_fadd_f64((__attribute__((address_space(1))) double*)p, (double)s1);
        __builtin_amdgcn_global_atomic_fadd_f64((__attribute__((address_space(1))) double*)(p + CMAX),
                                                (double)s2);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (tid < 4) flag[tid] = 0;
      __syncthreads();
      if (tid == 0)
        __hip_atomic_fetch_add(&c->cnt[blockIdx.x % 8][0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (tid < 8) {
        const unsigned target = (unsigned)it * (unsigned)((G - tid + 7) / 8);
        const long long t0 = wall_clock64();
        for (;;) {
          const bool done = ld_agent(&c->cnt[tid][0]) >= target;
          if (__builtin_amdgcn_ballot_w64(!done) == 0) break;
          __builtin_amdgcn_s_sleep(1);
          if (wall_clock64() - t0 > kSpinTicks) {
            if (tid == 0) flag[1] = 1;
            break;
          }
        }
      }
      __syncthreads();
      ok = flag[1] == 0;
      if (tid < ch) {
        double a[4], b[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          a[r] = ld_agent_d(&A->d[r][0][tid]);
          b[r] = ld_agent_d(&A->d[r][1][tid]);
        }
        tbl[tid] = a[0] + a[1] + a[2] + a[3];
        tbl[CMAX + tid] = b[0] + b[1] + b[2] + b[3];
      }
      __syncthreads();
    } else {
      u32x4* buf = &c->slot[it & 1][0][0];
      if (tid < ch) {
        const unsigned b1 = __float_as_uint(s1), b2 = __float_as_uint(s2), tag = (unsigned)it;
        st_wt_b128(buf, blockIdx.x * CMAX + tid, u32x4{b1, b2, tag, tag ^ b1 ^ b2});
      }
      // thread t: channel t % ch, workgroups g = t / ch, + NT / ch, ...
      const int cc = tid % ch, g0 = tid / ch, gs = NT / ch;
      double p1 = 0.0, p2 = 0.0;
      const long long t0 = wall_clock64();
      int fail = 0;
      for (int g = g0; g < G; g += gs) {
        u32x4 v = ld_wt_b128(buf, g * CMAX + cc);
        while (v[2] != (unsigned)it || (v[3] ^ v[2] ^ v[0] ^ v[1]) != 0u) {
          __builtin_amdgcn_s_sleep(1);
          if (wall_clock64() - t0 > kSpinTicks) {
            fail = 1;
            break;
          }
          v = ld_wt_b128(buf, g * CMAX + cc);
        }
        p1 += (double)__uint_as_float(v[0]);
        p2 += (double)__uint_as_float(v[1]);
      }
      red[0][tid] = p1;
      red[1][tid] = p2;
      if (fail) flag[1] = 1;
      __syncthreads();
      ok = flag[1] == 0;
      if (tid < ch) {
        double a = 0.0, b = 0.0;
        for (int i = 0; i < gs; ++i) {
          a += red[0][i * ch + tid];
          b += red[1][i * ch + tid];
        }
        tbl[tid] = a;
        tbl[CMAX + tid] = b;
      }
      __syncthreads();
    }
    // check: the expected total of s1 = x + g over the workgroups (x is the same on every
    // workgroup: same work, same thread)
    if (tid < ch && do_sums > 1) {
      double want = 0.0;
      for (int g = 0; g < G; ++g) want += (double)(x + (float)g);
      if (fabs(tbl[tid] - want) > 1e-3 * (double)G)
        __hip_atomic_fetch_add(&c->bad, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    x += (float)tbl[tid % CMAX] * 1e-30f;
  }
  if (tid == 0 && x == 12345.f) c->sink[blockIdx.x] = x;
}

template <int MODE>
static float run(Ctl* c, Acc* accs, int G, int iters, int work, int sums, int ch, unsigned* fail,
                 unsigned* bad) {
  CK(hipMemset(c, 0, sizeof(Ctl)));
  CK(hipMemset(accs, 0, sizeof(Acc) * NBAR));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  hipLaunchKernelGGL((bar_kernel<MODE>), dim3(G), dim3(NT), 0, 0, c, accs, iters, work, sums, ch);
  CK(hipGetLastError());
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipMemcpy(fail, &c->fail, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(bad, &c->bad, 4, hipMemcpyDeviceToHost));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms;
}

template <int MODE>
static float per_barrier(Ctl* c, Acc* accs, int G, int work, int ch, bool* badf) {
  const int B = NBAR;
  std::vector<float> t;
  for (int r = 0; r < 5; ++r) {
    unsigned f = 0, bd = 0;
    const float t1 = run<MODE>(c, accs, G, B, work, 1, ch, &f, &bd);
    if (f) *badf = true;
    const float t0 = run<MODE>(c, accs, G, B, work, -1, ch, &f, &bd);
    t.push_back((t1 - t0) * 1000.f / B);
  }
  // one checked run: every workgroup's totals are the exact expected sum
  unsigned f = 0, bd = 0;
  run<MODE>(c, accs, G, 200, work, 2, ch, &f, &bd);
  if (f || bd) *badf = true;
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  Ctl* c;
  Acc* accs;
  CK(hipMalloc(&c, sizeof(Ctl)));
  CK(hipMalloc(&accs, sizeof(Acc) * NBAR));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  std::printf("# BatchNorm barrier: fp64 atomics + sharded counter vs tagged slots (%s, %d CUs)\n\n",
              prop.name, prop.multiProcessorCount);
  std::printf("us per barrier (median of 5 launches of 2000 barriers, minus the work alone), 512-thread "
              "workgroups, one per CU. `microbench/bn_slots.hip`.\n\n");
  std::printf("| workgroups | channels | work | atom | slot | int | int1 | int2 |\n|---|---|---|---|---|---|---|---|\n");
  for (int G : {16, 64, 128, 256}) {
    for (int ch : {16, 64}) {
      for (int work : {0, 400}) {
        bool bad = false;
        bool bi = false, bi1 = false, ba = false, bs = false;
        const float a = per_barrier<ATOM>(c, accs, G, work, ch, &ba);
        const float s = per_barrier<SLOT>(c, accs, G, work, ch, &bs);
        const float q = per_barrier<INT>(c, accs, G, work, ch, &bi);
        const float q1 = per_barrier<INT1>(c, accs, G, work, ch, &bi1);
        bool bi2 = false;
        const float q2 = per_barrier<INT2>(c, accs, G, work, ch, &bi2);
        bad = ba || bs || bi || bi1 || bi2;
        std::printf("| %d | %d | %d | %.2f | %.2f | %.2f | %.2f | %.2f |%s%s%s%s%s\n", G, ch, work, a, s, q, q1, q2,
                    bi2 ? " int2-FAIL" : "",
                    ba ? " atom-FAIL" : "", bs ? " slot-FAIL" : "", bi ? " int-FAIL" : "",
                    bi1 ? " int1-FAIL" : "");
        std::fflush(stdout);
      }
    }
  }
  CK(hipFree(c));
  CK(hipFree(accs));
  return 0;
}
