// Optimizer and flat-parameter plumbing.
//
// Replaces TF's ApplyMomentum x152 + L2Loss x152 + AddN + AssignAdd(global_step)
// (resnet_model.py:85-99,120-122):
//   g'    = grad * grad_scale + wd * w          (d/dw of wd * sum 1/2 ||w||^2)
//   accum = momentum * accum + g'                (tf.train.MomentumOptimizer, non-Nesterov)
//   w    -= lr * accum
// in ONE launch over the flat fp32 master buffer, which also re-packs every conv
// kernel into the two bf16 layouts the MFMA kernels consume ([K][kh][kw][C] for
// forward, HWIO for dgrad).  The learning rate is evaluated on the device from
// the device-resident global_step with the reference's piecewise schedule
// (resnet_cifar_main.py:304-324, resnet_imagenet_main.py:306-329 incl. the
// step-0 quirk), so the whole training step can be captured in a hipGraph.
#include "common.h"
#include "kernels.h"
#include "optim.h"

namespace dtr {

__device__ __forceinline__ float lr_at(const LrSchedule& s, long step) {
  // The reference's hook feeds the rate computed after the *previous* run:
  // step 0 uses the initial value from begin(); step t>0 uses f(t-1).
  if (step <= 0) return s.init;
  const long t = step - 1;
  if (t < s.warm_steps) return s.warm_from + (s.warm_to - s.warm_from) * (float)t / (float)s.warm_steps;
  for (int i = 0; i < s.nb; ++i)
    if (t < s.bound[i]) return s.val[i];
  return s.val[s.nb];
}

constexpr int SEG_LDS_MAX = 640;   // segment tables cached in LDS up to this size (30 KB)

__device__ __forceinline__ int find_seg(const ParamSeg* segs, int nseg, long e) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (segs[mid].offset <= e) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}


// HWIO bf16 copy of element e (contiguous with e: the master IS HWIO order).
__device__ __forceinline__ void write_hwio(const ParamSeg& sg, long e, float w, bf16* bf) {
  if (sg.bf_hwio < 0) return;
  const long local = e - sg.offset;
  if (sg.kpad == sg.K) {
    bf[sg.bf_hwio + local] = (bf16)w;
  } else {
    const long row = local / sg.K, co = local - row * sg.K;
    bf[sg.bf_hwio + row * sg.kpad + co] = (bf16)w;
  }
}

// The update itself: 4 consecutive elements per thread (16-B loads / stores of
// w, grad, momentum; an 8-B store of the HWIO bf16 copy) with the parameter
// segment tracked incrementally per thread (elements only move forward) instead
// of a binary search per element.  The OHWI copy (a transpose) is ohwi_pack's.
__global__ void __launch_bounds__(256)
sgd_pack_kernel(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ mom,
                long n, LrSchedule sched, const long long* __restrict__ gstep, float momentum,
                float wd, float grad_scale, int use_momentum, const ParamSeg* __restrict__ segs,
                int nseg, bf16* __restrict__ bf, float* __restrict__ lr_out, int update) {
  // the segment table in LDS: one coalesced round trip per block instead of a binary
  // search of dependent global loads per thread (~8 for ResNet-50's 161 tensors)
  __shared__ ParamSeg sseg[SEG_LDS_MAX];
  const ParamSeg* S = segs;
  if (nseg <= SEG_LDS_MAX) {
    for (int i = threadIdx.x; i < nseg; i += blockDim.x) sseg[i] = segs[i];
    __syncthreads();
    S = sseg;
  }
  const float lr = update ? lr_at(sched, gstep ? (long)*gstep : 0L) : 0.f;
  if (update && lr_out && blockIdx.x == 0 && threadIdx.x == 0) *lr_out = lr;
  const long nv = (n + 3) / 4;
  const long stride = (long)gridDim.x * blockDim.x;
  long v = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (v >= nv) return;
  int sgi = find_seg(S, nseg, v * 4);
  for (; v < nv; v += stride) {
    const long e0 = v * 4;
    while (sgi + 1 < nseg && S[sgi + 1].offset <= e0) ++sgi;
    const ParamSeg& sg = S[sgi];
    const bool whole = e0 + 4 <= n && e0 + 4 <= sg.offset + sg.numel;
    if (whole) {
      f32x4 wv = *reinterpret_cast<const f32x4*>(w + e0);
      if (update) {
        const f32x4 gv = *reinterpret_cast<const f32x4*>(g + e0) * grad_scale + wd * wv;
        if (use_momentum) {
          const f32x4 acc = momentum * *reinterpret_cast<const f32x4*>(mom + e0) + gv;
          *reinterpret_cast<f32x4*>(mom + e0) = acc;
          wv -= lr * acc;
        } else {
          wv -= lr * gv;
        }
        *reinterpret_cast<f32x4*>(w + e0) = wv;
      }
      if (bf && sg.bf_hwio >= 0) {
        if (sg.kpad == sg.K && ((e0 - sg.offset) & 3) == 0) {
          bf16x4 h = {(bf16)wv[0], (bf16)wv[1], (bf16)wv[2], (bf16)wv[3]};
          *reinterpret_cast<bf16x4*>(bf + sg.bf_hwio + (e0 - sg.offset)) = h;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) write_hwio(sg, e0 + j, wv[j], bf);
        }
      }
    } else {   // a vector straddling a segment end (e.g. a 10-class bias) or the tail
      for (int j = 0; j < 4 && e0 + j < n; ++j) {
        const long e = e0 + j;
        const ParamSeg& sj = S[find_seg(S, nseg, e)];
        float wj = w[e];
        if (update) {
          const float gj = g[e] * grad_scale + wd * wj;
          if (use_momentum) {
            const float acc = momentum * mom[e] + gj;
            mom[e] = acc;
            wj -= lr * acc;
          } else {
            wj -= lr * gj;
          }
          w[e] = wj;
        }
        if (bf) write_hwio(sj, e, wj, bf);
      }
    }
  }
}

void sgd_update_pack(float* master, const float* grad, float* mom, long n, const LrSchedule& s,
                     const long long* gstep, float momentum, float wd, float grad_scale,
                     int use_momentum, const ParamSeg* segs, int nseg, bf16* bf, float* lr_out,
                     int update, hipStream_t st) {
  long blocks = ((n + 3) / 4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(sgd_pack_kernel, dim3((unsigned)blocks), dim3(256), 0, st, master, grad, mom,
                     n, s, gstep, momentum, wd, grad_scale, use_momentum, segs, nseg, bf, lr_out,
                     update);
  DTR_CHECK_LAUNCH();
}

// OHWI bf16 copies of every weight: a tiled transpose of the fp32 master
// ([tap*C + ci][co], HWIO) into [co][tap*cpad + ci] through LDS so both the
// reads (along co) and the writes (along tap*C + ci) are coalesced -- the per-
// element scattered 2-byte stores of the fused form were most of the optimizer
// launch's time on ImageNet.  tile0[s] = first tile of segment s (prefix over
// ceil(taps*C/64) x ceil(K/64) tiles; segments without an OHWI copy have 0 tiles).
__global__ void __launch_bounds__(256)
ohwi_pack_kernel(const float* __restrict__ w, const ParamSeg* __restrict__ segs,
                 const long long* __restrict__ tile0, int nseg, bf16* __restrict__ bf,
                 long long* gstep_inc) {
  __shared__ bf16 tile[64][66];
  __shared__ long long st0[SEG_LDS_MAX];
  __shared__ int seg_of_block;
  const long long b = blockIdx.x;
  // the step's global_step += 1 rides here (this kernel never reads it): one launch less
  if (gstep_inc != nullptr && b == 0 && threadIdx.x == 0) *gstep_inc += 1;
  int lo = 0;
  if (nseg <= SEG_LDS_MAX) {   // first-tile table in LDS (one coalesced round trip)
    for (int i = threadIdx.x; i < nseg; i += blockDim.x) st0[i] = tile0[i];
    __syncthreads();
    if (threadIdx.x == 0) {
      int l = 0, h = nseg - 1;
      while (l < h) {
        const int mid = (l + h + 1) >> 1;
        if (st0[mid] <= b) l = mid;
        else h = mid - 1;
      }
      seg_of_block = l;
    }
    __syncthreads();
    lo = seg_of_block;
  } else {
    int hi = nseg - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (tile0[mid] <= b) lo = mid;
      else hi = mid - 1;
    }
  }
  const ParamSeg& sg = segs[lo];
  const int taps = sg.kh * sg.kw;
  const int R = taps * sg.C;                 // HWIO rows (tap, ci)
  const int tc_n = (sg.K + 63) / 64;
  const int t = (int)(b - (nseg <= SEG_LDS_MAX ? st0[lo] : tile0[lo]));
  const int tr = t / tc_n, tcol = t - tr * tc_n;
  const int r0 = tr * 64, c0 = tcol * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {         // read rows r0+i, cols c0+tx (coalesced)
    const int r = r0 + i, co = c0 + tx;
    tile[i][tx] = (r < R && co < sg.K) ? (bf16)w[sg.offset + (long)r * sg.K + co] : (bf16)0.f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {         // write rows co = c0+i, cols r0+tx (coalesced)
    const int co = c0 + i, r = r0 + tx;
    if (co < sg.K && r < R) {
      const int tap = r / sg.C, ci = r - tap * sg.C;
      bf[sg.bf_ohwi + ((long)co * taps + tap) * sg.cpad + ci] = tile[tx][i];
    }
  }
}

void ohwi_pack(const float* master, const ParamSeg* segs, const long long* tile0, int nseg,
               long long total_tiles, bf16* bf, long long* gstep_inc, hipStream_t s) {
  if (total_tiles <= 0) {
    if (gstep_inc) step_increment(gstep_inc, s);
    return;
  }
  hipLaunchKernelGGL(ohwi_pack_kernel, dim3((unsigned)total_tiles), dim3(256), 0, s, master,
                     segs, tile0, nseg, bf, gstep_inc);
  DTR_CHECK_LAUNCH();
}

// The persistent step's optimizer in ONE launch, instead of the grouped slab reduce,
// sgd_pack and ohwi_pack (three dependent launches, ~31 us of a 0.87 ms CIFAR step,
// profiles/cifar_persist_bs128_kernels.md).  A weight is cut into TR (rows tap*C+ci)
// x TC (co) tiles of its HWIO master (host-chosen so a tile's slab loads are <= 8
// 16-byte loads per thread: 64x64 without slabs, 16x16 for 32 splits):
//   1. (slab mode) its split-K slabs ([split][co][tap*cslab+ci]) summed -- 16-byte
//      loads along (tap, ci), the slabs' contiguous axis; past 8 splits 4 thread groups
//      take every 4th split and their partials are added in group order, the grouped
//      reduce's order -- into LDS [co][r];
//   2. per element: g' = g*scale + wd*w, acc = momentum*acc + g', w -= lr*acc; the fp32
//      gradient (slab mode), master, momentum and the bf16 HWIO copy;
//   3. the bf16 tile transposed through LDS into the OHWI copy (written along ci).
// Other tensors (BN gamma/beta, biases) go in 1024-element chunks.  The rate comes from
// global_step; the last workgroup to finish (by ticket) does global_step += 1.
// World > 1 (optim.h): `pack` launches stop after the gradient (written as the bf16
// all-reduce input `gout`, or to grad), and the update launch then reads it back from
// `gin` (the all-reduced bf16).
// MODE 0: update (gradient from slabs / grad); 1: pack; 2: update from gin.
template <int MODE>
__global__ void __launch_bounds__(256)
sgd_tiles_kernel(float* __restrict__ w, float* __restrict__ g, float* __restrict__ mom,
                 LrSchedule sched, long long* gstep, float momentum, float wd,
                 float grad_scale, int use_momentum, const ParamSeg* __restrict__ segs,
                 const OptWork* __restrict__ work, const int* __restrict__ blk_seg,
                 bf16* __restrict__ bf, float* __restrict__ lr_out, unsigned* ticket,
                 const bf16* __restrict__ gin, bf16* __restrict__ gout) {
  constexpr bool pack = MODE == 1, from_gin = MODE == 2;
  __shared__ float gt[64][65];   // summed gradient tile [co][r]
  __shared__ bf16 bt[64][66];    // updated bf16 tile [r][co]
  __shared__ f32x4 red[256];     // split-group partials
  __shared__ float lr_s;
  const int tid = threadIdx.x;
  const int si = blk_seg[blockIdx.x];
  const ParamSeg sg = segs[si];
  const OptWork ow = work[si];
  if (tid == 0) {
    const float lr0 = lr_at(sched, (long)*gstep);
    lr_s = lr0;
    if (lr_out && blockIdx.x == 0) *lr_out = lr0;
  }
  const int t = (int)((long long)blockIdx.x - ow.tile0);
  if (ow.tiled) {
    const int taps = sg.kh * sg.kw, C = sg.C, K = sg.K, R = taps * C;
    const int TR = ow.tr, TC = ow.tc;
    const int tc_n = (K + TC - 1) / TC;
    const int r0 = (t / tc_n) * TR, c0 = (t - (t / tc_n) * tc_n) * TC;
    const int nr = min(TR, R - r0), nc = min(TC, K - c0);   // valid extent
    const bool slab = ow.part != nullptr;
    const int lc = __builtin_ctz(TC);                         // TC: a power of two
    // this thread's elements' master, momentum and (no slab) gradient, loaded before
    // the slab sums so the two rounds of loads overlap (TR * TC <= 16 x 256)
    constexpr int EPT = 16;
    float wr[EPT], mr[EPT], gr[EPT];
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const int q = tid + j * 256, rl = q >> lc, cl = q & (TC - 1);
      wr[j] = mr[j] = gr[j] = 0.f;
      if (q < TR * TC && rl < nr && cl < nc) {
        const long e = sg.offset + (long)(r0 + rl) * K + c0 + cl;
        if constexpr (!pack) {
          wr[j] = w[e];
          if (use_momentum) mr[j] = mom[e];
        }
        if (!slab) gr[j] = from_gin ? (float)gin[e] : g[e];
      }
    }
    if (slab) {
      // slab columns: the tile's rows (cslab == C: column n = row r, nr % 4 == 0) or,
      // for padded rows (the stem: C = 3 in rows of cslab; one row tile), all of them
      const int cs = ow.cslab;
      const bool padded = cs != C;
      const long NT = (long)taps * cs;
      const long stride = (long)ow.kslab * NT;    // one split's slab
      const int n0 = padded ? 0 : r0;
      const int ncol4 = padded ? (int)(NT >> 2) : (nr >> 2);
      const int U = nc * ncol4;                  // float4 units of the tile
      // the grouped reduce's summation order (conv_wgrad.hip, WGR_WIDE_MAX): splits in
      // sequence up to 8, else 4 interleaved groups added in group order -- so a step
      // with and without an all-reduce in between agree bit for bit (G*U <= 256: host)
      const int G = ow.splits > 8 ? 4 : 1;
      auto scatter = [&](const f32x4& a, int col, int c4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n0 + c4 + j;
          if (padded) {
            const int tap = n / cs, ci = n - tap * cs;
            if (ci < C) gt[col][tap * C + ci] = a[j];
          } else {
            gt[col][c4 + j] = a[j];
          }
        }
      };
      for (int q = tid; q < G * U; q += 256) {
        const int u = q % U, gi = q / U;
        const int col = u / ncol4, c4 = (u - col * ncol4) * 4;
        const float* src = ow.part + (long)(c0 + col) * NT + n0 + c4;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        int s = gi;
        for (; s + 3 * G < ow.splits; s += 4 * G) {   // 4 loads in flight, order kept
          f32x4 v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            v[j] = *reinterpret_cast<const f32x4*>(src + (long)(s + j * G) * stride);
#pragma unroll
          for (int j = 0; j < 4; ++j) acc += v[j];
        }
        for (; s < ow.splits; s += G) acc += *reinterpret_cast<const f32x4*>(src + (long)s * stride);
        if (G == 1) scatter(acc, col, c4);
        else red[gi * U + u] = acc;
      }
      if (G > 1) {
        __syncthreads();
        for (int u = tid; u < U; u += 256) {
          f32x4 acc = red[u];
          for (int gi = 1; gi < G; ++gi) acc += red[gi * U + u];
          scatter(acc, u / ncol4, (u % ncol4) * 4);
        }
      }
    }
    __syncthreads();         // gt and lr_s
    const float lr = lr_s;
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const int q = tid + j * 256, rl = q >> lc, cl = q & (TC - 1);
      if (q < TR * TC && rl < nr && cl < nc) {
        const int r = r0 + rl, co = c0 + cl;
        const long e = sg.offset + (long)r * K + co;
        float gv = gr[j];
        if (slab) {
          gv = gt[cl][rl];
          g[e] = gv;
        } else if constexpr (from_gin) {
          g[e] = gv;
        }
        if constexpr (pack) {
          if (gout) gout[e] = (bf16)gv;
          continue;
        }
        float wv = wr[j];
        gv = gv * grad_scale + wd * wv;
        if (use_momentum) {
          const float a = momentum * mr[j] + gv;
          mom[e] = a;
          wv -= lr * a;
        } else {
          wv -= lr * gv;
        }
        w[e] = wv;
        if (sg.bf_hwio >= 0) bf[sg.bf_hwio + (long)r * sg.kpad + co] = (bf16)wv;
        bt[rl][cl] = (bf16)wv;
      }
    }
    if (sg.bf_ohwi >= 0 && !pack) {
      __syncthreads();
      for (int q = tid; q < TR * TC; q += 256) {   // along r: the OHWI copy's ci runs
        const int cl = q / TR, rl = q - cl * TR;
        if (rl < nr && cl < nc) {
          const int r = r0 + rl, co = c0 + cl;
          const int tap = r / C, ci = r - tap * C;
          bf[sg.bf_ohwi + ((long)co * taps + tap) * sg.cpad + ci] = bt[rl][cl];
        }
      }
    }
  } else {
    __syncthreads();
    const float lr = lr_s;
    const long base = (long)t * 1024;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long l = base + j * 256 + tid;
      if (l < sg.numel) {
        const long e = sg.offset + l;
        const float g0 = from_gin ? (float)gin[e] : g[e];
        if constexpr (from_gin) g[e] = g0;
        if constexpr (pack) {
          if (gout) gout[e] = (bf16)g0;
          continue;
        }
        float wv = w[e];
        const float gv = g0 * grad_scale + wd * wv;
        if (use_momentum) {
          const float a = momentum * mom[e] + gv;
          mom[e] = a;
          wv -= lr * a;
        } else {
          wv -= lr * gv;
        }
        w[e] = wv;
      }
    }
  }
  // global_step += 1 once every workgroup has read it: thread 0 consumed its read (lr_s)
  // before it takes the ticket, so a relaxed ticket orders it -- no fence: an agent-scope
  // release/acquire writes back and invalidates the L2 per workgroup (613 of them: the
  // launch took 54 us with __threadfence + acq_rel); the last one re-arms the ticket
  if (tid == 0 && !pack && ticket != nullptr) {   // (null: an early bucket's update, no step)
    const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      *gstep += 1;
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

void sgd_tiles(float* master, float* grad, float* mom, const LrSchedule& s, long long* gstep,
               float momentum, float wd, float grad_scale, int use_momentum,
               const ParamSeg* segs, const OptWork* work, const int* blk_seg, int nblocks,
               bf16* bf, float* lr_out, unsigned* ticket, const bf16* gin, bf16* gout, int pack,
               hipStream_t st) {
  if (nblocks <= 0) return;
#define DTR_SGD_TILES(M)                                                                        \
  hipLaunchKernelGGL(sgd_tiles_kernel<M>, dim3((unsigned)nblocks), dim3(256), 0, st, master, grad,  \
                     mom, s, gstep, momentum, wd, grad_scale, use_momentum, segs, work, blk_seg, bf, \
                     lr_out, ticket, gin, gout)
  if (pack) DTR_SGD_TILES(1);
  else if (gin) DTR_SGD_TILES(2);
  else DTR_SGD_TILES(0);
#undef DTR_SGD_TILES
  DTR_CHECK_LAUNCH();
}

__global__ void step_incr_kernel(long long* gstep) {
  if (threadIdx.x == 0) *gstep += 1;
}
void step_increment(long long* gstep, hipStream_t s) {
  hipLaunchKernelGGL(step_incr_kernel, dim3(1), dim3(64), 0, s, gstep);
  DTR_CHECK_LAUNCH();
}

// 1/2 * sum v^2 -- two-stage, fixed order (deterministic).
__global__ void __launch_bounds__(256) l2_part_kernel(const float* __restrict__ v, long n,
                                                      float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    s += v[i] * v[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}
__global__ void __launch_bounds__(256) l2_final_kernel(const float* __restrict__ part, int np,
                                                       float* out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < np; i += 256) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *out = 0.5f * (red[0] + red[1] + red[2] + red[3]);
}

static constexpr int L2_BLOCKS = 512;
int l2_workspace_floats() { return L2_BLOCKS; }

void l2_half_sum(const float* v, long n, float* ws, float* out, hipStream_t s) {
  hipLaunchKernelGGL(l2_part_kernel, dim3(L2_BLOCKS), dim3(256), 0, s, v, n, ws);
  hipLaunchKernelGGL(l2_final_kernel, dim3(1), dim3(256), 0, s, ws, L2_BLOCKS, out);
  DTR_CHECK_LAUNCH();
}

__global__ void fill_kernel(float* p, long n, float a) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    p[i] = a;
}
void fill_f32(float* p, long n, float a, hipStream_t s) {
  long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(fill_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, n, a);
  DTR_CHECK_LAUNCH();
}

__global__ void cast_f2b_kernel(const float* a, bf16* b, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    b[i] = (bf16)a[i];
}
__global__ void cast_b2f_kernel(const bf16* a, float* b, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x)
    b[i] = (float)a[i];
}
void cast_f32_bf16(const float* a, bf16* b, long n, hipStream_t s) {
  long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(cast_f2b_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, b, n);
  DTR_CHECK_LAUNCH();
}
void cast_bf16_f32(const bf16* a, float* b, long n, hipStream_t s) {
  long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(cast_b2f_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, b, n);
  DTR_CHECK_LAUNCH();
}

}  // namespace dtr
