// Python bindings + native static-plan executor.
//
// The reference runs its static TF graph through TF's C++ executor
// (MonitoredTrainingSession -> session.run(train_op)).  Here the
// ResNet training step is likewise static, so it is recorded ONCE into a
// `Plan`: a vector of launch closures with all pointers/shapes bound.  Running a
// segment of the plan is a tight native loop of hipLaunchKernel calls on the
// given stream (no Python per op); the whole step can additionally be captured
// into a hipGraph (train/engine.py) which removes the host launch cost.
//
// Every op is exposed twice from one definition: as an immediate call
// (`_C.conv_gemm(..., stream)`, used by ops/functional.py and the tests) and as
// a plan recorder (`plan.conv_gemm(...)`).  Device pointers travel as Python
// ints (tensor.data_ptr()); no torch headers are needed, which keeps this
// extension small and fast to build.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "comm.h"
#include "data.h"
#include "kernels.h"
#include "optim.h"

namespace py = pybind11;
using namespace dtr;

typedef uintptr_t ptr_t;
typedef std::function<void(hipStream_t)> Launch;

template <typename T>
static inline T* P(ptr_t p) {
  return reinterpret_cast<T*>(p);
}
static inline hipStream_t S(ptr_t s) { return reinterpret_cast<hipStream_t>(s); }

static ConvGeom geom_from(const std::vector<int>& v) {
  if (v.size() != 11) throw std::invalid_argument("geom needs 11 ints: N,H,W,C,Ho,Wo,K,kh,kw,stride,pad");
  return ConvGeom{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[9], v[10]};
}

// Split-K workspace a plan owns per stream (fp32 slice slabs + last-arriver tile counters
// of the split-K conv_gemm loops).  Sized while the plan's conv ops are recorded
// (conv_gemm_splitk_need), so a running step never allocates; ops of one stream run in
// stream order and share it, ops of different streams never do.
struct PlanSplitK {
  float* part = nullptr;
  size_t bytes = 0;
  unsigned* cnt = nullptr;
  size_t cnt_n = 0;
  void reserve(size_t b, size_t tiles) {
    if (b <= bytes && tiles <= cnt_n) return;
    (void)hipDeviceSynchronize();   // recording after a run: nothing may still read the old ones
    if (b > bytes) {
      void* p = nullptr;
      if (hipMalloc(&p, b) != hipSuccess) throw std::runtime_error("split-K workspace: hipMalloc failed");
      (void)hipFree(part);
      part = static_cast<float*>(p);
      bytes = b;
    }
    if (tiles > cnt_n) {
      void* p = nullptr;
      if (hipMalloc(&p, tiles * sizeof(unsigned)) != hipSuccess ||
          hipMemset(p, 0, tiles * sizeof(unsigned)) != hipSuccess)
        throw std::runtime_error("split-K counters: hipMalloc failed");
      (void)hipFree(cnt);
      cnt = static_cast<unsigned*>(p);
      cnt_n = tiles;
    }
  }
  ~PlanSplitK() {
    (void)hipFree(part);
    (void)hipFree(cnt);
  }
};
// set while a plan records an op: the workspace of the plan's current stream
static thread_local PlanSplitK* g_rec_splitk = nullptr;

// ---------------------------------------------------------------- op makers
// Partials a consumer prologue (bn_prefin_table / bn_prefin_sums, bn_fused.h)
// combines for C channels: C/4 float4 groups, PFIN_ROUNDS rounds of PFIN_ITEMS.
static int pfin_cap(int C) {
  if (C < 4 || C > 128 || (C & (C - 1)) != 0) return 0;
  return 8 * 2 * 1024 / C;
}

static Launch mk_conv_gemm(int mode, ptr_t a, ptr_t b, ptr_t out, ptr_t out_f32, ptr_t residual,
                           ptr_t pre_scale, ptr_t pre_shift, ptr_t bias, int nbias,
                           ptr_t stat_part, int accumulate, std::vector<int> geom,
                           std::vector<ptr_t> bnb, std::vector<ptr_t> fin,
                           std::vector<ptr_t> bfin, std::vector<ptr_t> pfin,
                           std::vector<ptr_t> abwd, float momentum, float eps,
                           int update_moving) {
  GemmArgs g{};
  g.a = P<const bf16>(a);
  g.b = P<const bf16>(b);
  g.out = P<bf16>(out);
  g.out_f32 = P<float>(out_f32);
  g.residual = P<const bf16>(residual);
  g.pre_scale = P<const float>(pre_scale);
  g.pre_shift = P<const float>(pre_shift);
  g.bias = P<const float>(bias);
  g.nbias = nbias;
  g.stat_part = P<float>(stat_part);
  g.accumulate = accumulate;
  if (!bnb.empty()) {  // [x, mean, rstd, scale, shift, part]: fused BN-ReLU backward reduce
    if (bnb.size() != 6) throw std::invalid_argument("bnb needs 6 pointers");
    if (mode != MODE_DGRAD) throw std::invalid_argument("bnb is dgrad-only");
    g.bnb_x = P<const bf16>(bnb[0]);
    g.bnb_mean = P<const float>(bnb[1]);
    g.bnb_rstd = P<const float>(bnb[2]);
    g.bnb_scale = P<const float>(bnb[3]);
    g.bnb_shift = P<const float>(bnb[4]);
    g.bnb_part = P<float>(bnb[5]);
  }
  if (fin.size() == 1) {  // [acc]: STATS into the fp64 accumulator replicas (kernels.h)
    if (stat_part == 0) throw std::invalid_argument("stat acc requires stat_part");
    g.stat_acc = P<double>(fin[0]);
    fin.clear();
  }
  if (bfin.size() == 1) {  // [acc]: BNB sums into the fp64 accumulator replicas
    if (bnb.empty()) throw std::invalid_argument("bnb acc requires bnb");
    g.bnb_acc = P<double>(bfin[0]);
    bfin.clear();
  }
  if (!fin.empty()) {  // [counters, gamma, beta, mmean, mvar, mean, rstd, scale, shift, gpart,
                       //  group, groups_only]
    if (fin.size() != 12) throw std::invalid_argument("fin needs 12 entries");
    if (stat_part == 0) throw std::invalid_argument("fin requires stat_part");
    g.fin = BnFwdFin{P<unsigned>(fin[0]), P<const float>(fin[1]), P<const float>(fin[2]),
                     P<float>(fin[3]), P<float>(fin[4]), P<float>(fin[5]), P<float>(fin[6]),
                     P<float>(fin[7]), P<float>(fin[8]), momentum, eps, update_moving,
                     P<float>(fin[9]), (int)fin[10], (int)fin[11]};
  }
  if (!bfin.empty()) {  // [counters, gamma, rstd, dgamma, dbeta, coef, gpart, group, groups_only]
    if (bfin.size() != 9) throw std::invalid_argument("bfin needs 9 entries");
    if (bnb.empty()) throw std::invalid_argument("bfin requires bnb");
    g.bfin = BnBwdFin{P<unsigned>(bfin[0]), P<const float>(bfin[1]), P<const float>(bfin[2]),
                      P<float>(bfin[3]), P<float>(bfin[4]), P<float>(bfin[5]),
                      P<float>(bfin[6]), (int)bfin[7], (int)bfin[8]};
  }
  if (!pfin.empty()) {  // [part, cnt, rows_per, M, gamma, beta, mean, rstd, scale, shift, mmean, mvar]
    if (pfin.size() != 12) throw std::invalid_argument("pfin needs 12 entries");
    if (pre_scale == 0) throw std::invalid_argument("pfin requires the PRE prologue");
    // cnt == -1: part is a [BN_ACC_REP][2][C] fp64 accumulator (acc mode)
    const bool acc = (int)pfin[1] == -1;
    g.pfin = BnPreFin{acc ? nullptr : P<const float>(pfin[0]), acc ? 1 : (int)pfin[1],
                      acc ? P<const double>(pfin[0]) : nullptr, (int)pfin[2], (int)pfin[3],
                      P<const float>(pfin[4]), P<const float>(pfin[5]), P<float>(pfin[6]),
                      P<float>(pfin[7]), P<float>(pfin[8]), P<float>(pfin[9]),
                      P<float>(pfin[10]), P<float>(pfin[11]), momentum, eps, update_moving};
  }
  if (!abwd.empty()) {  // [x, add, mean, rstd, scale, shift, gamma, part, cnt, a_out, dgamma,
                       //  dbeta, coef]
    if (abwd.size() != 13) throw std::invalid_argument("abwd needs 13 entries");
    if (mode != MODE_DGRAD) throw std::invalid_argument("abwd is dgrad-only");
    const bool acc = (int)abwd[8] == -1;   // part is a fp64 accumulator (acc mode)
    g.abwd = BnBwdPre{P<const bf16>(abwd[0]), P<const bf16>(abwd[1]), P<const float>(abwd[2]),
                      P<const float>(abwd[3]), P<const float>(abwd[4]), P<const float>(abwd[5]),
                      P<const float>(abwd[6]), acc ? nullptr : P<const float>(abwd[7]),
                      acc ? 1 : (int)abwd[8], acc ? P<const double>(abwd[7]) : nullptr,
                      P<bf16>(abwd[9]), P<float>(abwd[10]), P<float>(abwd[11]),
                      P<float>(abwd[12])};
  }
  if (out == 0 && out_f32 == 0) throw std::invalid_argument("conv_gemm: out or out_f32 needed");
  g.g = geom_from(geom);
  const ConvGeom& c = g.g;
  const int taps = c.kh * c.kw;
  if (mode == MODE_FWD) {
    g.M = c.N * c.Ho * c.Wo;
    g.Ncol = c.K;
    g.Kdim = taps * c.C;
    if (c.C % 8) throw std::invalid_argument("conv fwd: C must be a multiple of 8");
  } else {
    g.M = c.N * c.H * c.W;
    g.Ncol = c.C;
    g.Kdim = taps * c.K;
    if (c.K % 8) throw std::invalid_argument("conv dgrad: K must be a multiple of 8");
  }
  if (g.Ncol % 16) throw std::invalid_argument("conv: output channels must be a multiple of 16");
  if ((pre_scale != 0) && mode != MODE_FWD)
    throw std::invalid_argument("fused BN+ReLU prologue is forward-only");
  if (g.abwd.x != nullptr) {
    if (conv_direct_covers(g, mode)) {
      const int C = c.K;   // A channels of the dgrad
      if (g.abwd.acc == nullptr && (g.abwd.cnt < 0 || g.abwd.cnt > pfin_cap(C)))   // 0: coef precomputed
        throw std::invalid_argument("abwd: partial count exceeds the prologue bound");
    } else {
      throw std::invalid_argument("abwd: the fused BN-backward prologue needs the direct 3x3 "
                                  "dgrad (CIFAR shapes)");
    }
  }
  if (g.pfin.cnt > 0 && g.pfin.acc == nullptr) {
    const int C = c.C;   // PRE is forward-only: the A channels
    if (g.pfin.cnt > pfin_cap(C))
      throw std::invalid_argument("pfin: C must be a power of two in [4, 128] and cnt <= "
                                  "PFIN_ITEMS*PFIN_ROUNDS*1024/C");
  }
  // In-kernel finalize bounds (conv_epilogue.h combines): every level's item count
  // must fit one round of loads, cnt <= (256 / BN) * FIN_UNROLL.
  for (int which = 0; which < 2; ++which) {
    const bool on = which == 0 ? g.fin.counters != nullptr : g.bfin.counters != nullptr;
    if (!on) continue;
    const int grp = which == 0 ? g.fin.group : g.bfin.group;
    const int bm = conv_gemm_bm(g.M, g.Ncol), bn = conv_gemm_bn(g.M, g.Ncol);
    const int T = (g.M + bm - 1) / bm, cap = (256 / bn) * 8;
    const bool ok = grp == 0 ? T <= cap : (grp <= cap && (T + grp - 1) / grp <= cap);
    if (!ok || (grp != 0 && (which == 0 ? g.fin.gpart : g.bfin.gpart) == nullptr))
      throw std::invalid_argument("fused BN finalize: tile count exceeds the combine bound");
  }
  if (g_rec_splitk != nullptr) {   // a plan op: its stream's workspace, sized now
    size_t tiles = 0;
    const size_t need = conv_gemm_splitk_need(g, mode, &tiles);
    if (need > 0) {
      PlanSplitK* ws = g_rec_splitk;
      ws->reserve(need, tiles);
      return [g, mode, ws](hipStream_t s) {
        GemmArgs a = g;
        a.sk_part = ws->part;
        a.sk_cnt = ws->cnt;
        conv_gemm(a, mode, s);
      };
    }
  }
  return [g, mode](hipStream_t s) { conv_gemm(g, mode, s); };
}

// [dz, w, x, add, out, mean, rstd, scale, shift, coef, bacc]: bn_dgrad1x1.hip
static Launch mk_bnd1x1(int mode, std::vector<ptr_t> p, int M, int C, int K) {
  if (p.size() != 11) throw std::invalid_argument("bnd1x1 needs 11 pointers");
  if (!bnd1x1_covers(M, C, K))
    throw std::invalid_argument("bnd1x1: shape not covered (K in 64..512, C = 64 / 128 or a multiple of 256, resident weights <= 128 VGPRs, M % row tile)");
  if (mode < 0 || mode > 2) throw std::invalid_argument("bnd1x1 mode: 0 sums, 1 apply, 2 store + sums");
  if (mode != 1 && p[10] == 0) throw std::invalid_argument("bnd1x1 sums need bacc");
  if (mode >= 1 && p[4] == 0) throw std::invalid_argument("bnd1x1 apply / store need out");
  if (mode == 1 && p[9] == 0) throw std::invalid_argument("bnd1x1 apply needs coef");
  BndArgs a{P<const bf16>(p[0]), P<const bf16>(p[1]), P<const bf16>(p[2]), P<const bf16>(p[3]),
            P<bf16>(p[4]), P<const float>(p[5]), P<const float>(p[6]), P<const float>(p[7]),
            P<const float>(p[8]), P<const float>(p[9]), P<double>(p[10]), M, C, K};
  return [a, mode](hipStream_t s) { bnd1x1(a, mode, s); };
}

// [x, w, res, out, pre_scale, pre_shift, stat_acc]; pfin = conv_gemm's 12-entry list in
// accumulator mode (cnt == -1) or empty: bn_fwd1x1.hip
static Launch mk_bnf1x1(std::vector<ptr_t> p, std::vector<ptr_t> pfin, int M, int C, int K,
                        float momentum, float eps, int update_moving) {
  if (p.size() != 7) throw std::invalid_argument("bnf1x1 needs 7 pointers");
  if (!bnf1x1_covers(M, C, K))
    throw std::invalid_argument("bnf1x1: needs K in {64, 128, 256}, C % 256 == 0, M % row tile == 0");
  if (p[3] == 0 || p[1] == 0 || p[0] == 0) throw std::invalid_argument("bnf1x1: x, w, out needed");
  BnfArgs a{};
  a.x = P<const bf16>(p[0]);
  a.w = P<const bf16>(p[1]);
  a.res = P<const bf16>(p[2]);
  a.out = P<bf16>(p[3]);
  a.pre_scale = P<const float>(p[4]);
  a.pre_shift = P<const float>(p[5]);
  a.stat_acc = P<double>(p[6]);
  a.M = M;
  a.C = C;
  a.K = K;
  if (!pfin.empty()) {
    if (pfin.size() != 12 || (int)pfin[1] != -1)
      throw std::invalid_argument("bnf1x1: pfin must be the 12-entry accumulator-mode list");
    a.pfin = BnPreFin{nullptr, 1, P<const double>(pfin[0]), (int)pfin[2], (int)pfin[3],
                      P<const float>(pfin[4]), P<const float>(pfin[5]), P<float>(pfin[6]),
                      P<float>(pfin[7]), P<float>(pfin[8]), P<float>(pfin[9]),
                      P<float>(pfin[10]), P<float>(pfin[11]), momentum, eps, update_moving};
  }
  if ((a.pre_scale == nullptr) != (a.pre_shift == nullptr))
    throw std::invalid_argument("bnf1x1: pre_scale and pre_shift together");
  return [a](hipStream_t s) { bnf1x1(a, s); };
}

static Launch mk_conv_wgrad(ptr_t dy, ptr_t x, ptr_t pre_scale, ptr_t pre_shift, ptr_t part,
                            std::vector<int> geom, int splits, int px_per_split) {
  WgradArgs w{};
  w.dy = P<const bf16>(dy);
  w.x = P<const bf16>(x);
  w.pre_scale = P<const float>(pre_scale);
  w.pre_shift = P<const float>(pre_shift);
  w.part = P<float>(part);
  w.g = geom_from(geom);
  w.splits = splits;
  w.px_per_split = px_per_split;
  if (w.g.C % 8 || w.g.K % 16) throw std::invalid_argument("wgrad: C%8 and K%16 required");
  if (px_per_split % 64) throw std::invalid_argument("wgrad: px_per_split % 64");
  return [w](hipStream_t s) { conv_wgrad(w, s); };
}

static Launch mk_wgrad_reduce(ptr_t part, ptr_t grad, int splits, int K, int K_valid, int taps,
                              int C, int C_valid, float scale, int accumulate) {
  return [=](hipStream_t s) {
    wgrad_reduce(P<const float>(part), P<float>(grad), splits, K, K_valid, taps, C, C_valid, scale,
                 accumulate, s);
  };
}

static Launch mk_wgrad_reduce_grouped(ptr_t descs, int nd, long long total_chunks, float scale) {
  return [=](hipStream_t s) {
    wgrad_reduce_grouped(P<const WgReduceDesc>(descs), nd, total_chunks, scale, s);
  };
}

static Launch mk_bn_finalize(ptr_t part, int tiles, int tile_rows, int M, int C, ptr_t gamma,
                             ptr_t beta, ptr_t mmean, ptr_t mvar, float momentum, float eps,
                             int update_moving, ptr_t mean, ptr_t rstd, ptr_t scale,
                             ptr_t shift) {
  if (tiles == -1)   // part is a [BN_ACC_REP][2][C] fp64 accumulator (acc mode)
    return [=](hipStream_t s) {
      bn_finalize_acc(P<const double>(part), M, C, P<const float>(gamma), P<const float>(beta),
                      P<float>(mmean), P<float>(mvar), momentum, eps, update_moving,
                      P<float>(mean), P<float>(rstd), P<float>(scale), P<float>(shift), s);
    };
  return [=](hipStream_t s) {
    bn_finalize(P<const float>(part), tiles, tile_rows, M, C, P<const float>(gamma),
                P<const float>(beta), P<float>(mmean), P<float>(mvar), momentum, eps,
                update_moving, P<float>(mean), P<float>(rstd), P<float>(scale), P<float>(shift),
                s);
  };
}

static Launch mk_bn_eval(ptr_t gamma, ptr_t beta, ptr_t mm, ptr_t mv, float eps, int C,
                         ptr_t scale, ptr_t shift) {
  return [=](hipStream_t s) {
    bn_scale_shift_eval(P<const float>(gamma), P<const float>(beta), P<const float>(mm),
                        P<const float>(mv), eps, C, P<float>(scale), P<float>(shift), s);
  };
}

static Launch mk_bn_stats(ptr_t x, int M, int C, ptr_t part) {
  if (C % 8 || C > 2048) throw std::invalid_argument("bn_stats: C%8==0 and C<=2048");
  return [=](hipStream_t s) { bn_stats(P<const bf16>(x), M, C, P<float>(part), s); };
}

static Launch mk_bn_bwd_reduce(ptr_t dy, ptr_t x, ptr_t mean, ptr_t rstd, ptr_t scale,
                               ptr_t shift, int M, int C, ptr_t part) {
  if (C % 8 || C > 2048) throw std::invalid_argument("bn bwd: C%8==0 and C<=2048");
  return [=](hipStream_t s) {
    bn_relu_bwd_reduce(P<const bf16>(dy), P<const bf16>(x), P<const float>(mean),
                       P<const float>(rstd), P<const float>(scale), P<const float>(shift), M, C,
                       P<float>(part), nullptr, s);
  };
}

static Launch mk_bn_bwd_finalize(ptr_t part, int tiles, int M, int C, ptr_t gamma, ptr_t rstd,
                                 ptr_t dgamma, ptr_t dbeta, ptr_t coef) {
  if (tiles == -1)   // part is a [BN_ACC_REP][2][C] fp64 accumulator (acc mode)
    return [=](hipStream_t s) {
      bn_bwd_finalize_acc(P<const double>(part), M, C, P<const float>(gamma),
                          P<const float>(rstd), P<float>(dgamma), P<float>(dbeta), P<float>(coef),
                          s);
    };
  return [=](hipStream_t s) {
    bn_bwd_finalize(P<const float>(part), tiles, M, C, P<const float>(gamma),
                    P<const float>(rstd), P<float>(dgamma), P<float>(dbeta), P<float>(coef), s);
  };
}

static Launch mk_bn_bwd_apply(ptr_t dy, ptr_t x, ptr_t mean, ptr_t rstd, ptr_t scale,
                              ptr_t shift, ptr_t coef, ptr_t add, ptr_t dx, int M, int C) {
  return [=](hipStream_t s) {
    bn_relu_bwd_apply(P<const bf16>(dy), P<const bf16>(x), P<const float>(mean),
                      P<const float>(rstd), P<const float>(scale), P<const float>(shift),
                      P<const float>(coef), P<const bf16>(add), P<bf16>(dx), M, C, s);
  };
}

static Launch mk_bn_relu_apply(ptr_t x, ptr_t scale, ptr_t shift, ptr_t y, int M, int C) {
  return [=](hipStream_t s) {
    bn_relu_apply(P<const bf16>(x), P<const float>(scale), P<const float>(shift), P<bf16>(y), M,
                  C, s);
  };
}

static Launch mk_bn_relu_apply_acc(ptr_t x, ptr_t y, int M, int C, ptr_t acc, ptr_t gamma,
                                   ptr_t beta, ptr_t mmean, ptr_t mvar, float momentum, float eps,
                                   int update_moving, ptr_t mean, ptr_t rstd, ptr_t scale,
                                   ptr_t shift) {
  return [=](hipStream_t s) {
    bn_relu_apply_acc(P<const bf16>(x), P<bf16>(y), M, C, P<const double>(acc),
                      P<const float>(gamma), P<const float>(beta), P<float>(mmean), P<float>(mvar),
                      momentum, eps, update_moving, P<float>(mean), P<float>(rstd), P<float>(scale),
                      P<float>(shift), s);
  };
}

static Launch mk_bnrelu_avgpool(ptr_t x, ptr_t scale, ptr_t shift, ptr_t pooled, int N, int HW,
                                int C) {
  if (C % 8 || C > 2048) throw std::invalid_argument("avgpool: C%8==0 and C<=2048");
  return [=](hipStream_t s) {
    bnrelu_avgpool(P<const bf16>(x), P<const float>(scale), P<const float>(shift),
                   P<bf16>(pooled), N, HW, C, s);
  };
}

static Launch mk_avgpool_bwd(ptr_t dp, ptr_t dx, int N, int HW, int C) {
  return [=](hipStream_t s) { avgpool_bwd(P<const bf16>(dp), P<bf16>(dx), N, HW, C, s); };
}

static Launch mk_softmax_xent(ptr_t logits, int ld, ptr_t labels, int N, int classes,
                              ptr_t loss_sum, ptr_t correct, ptr_t dlogits, ptr_t dbias,
                              float grad_scale, ptr_t probs, ptr_t ws) {
  return [=](hipStream_t s) {
    softmax_xent(P<const float>(logits), ld, P<const int>(labels), N, classes, P<float>(loss_sum),
                 P<float>(correct), P<bf16>(dlogits), P<float>(dbias), grad_scale,
                 P<float>(probs), P<float>(ws), s);
  };
}

static Launch mk_softmax_xent_reduce(ptr_t ws, int ld, int N, int classes, ptr_t loss_sum,
                                     ptr_t correct, ptr_t dbias) {
  return [=](hipStream_t s) {
    softmax_xent_reduce(P<const float>(ws), ld, N, classes, P<float>(loss_sum), P<float>(correct),
                        P<float>(dbias), s);
  };
}

// head_fused(x, bn=[acc, gamma, beta, mmean, mvar, mean, rstd, scale, shift], momentum, eps,
//            update_moving, w_hwio, bias, labels, shape=[N, HW, C, classes, kpad], grad_scale,
//            out=[pooled, dlogits, ws, dact, bacc])
static Launch mk_head_fused(ptr_t x, std::vector<ptr_t> bn, float momentum, float eps,
                            int update_moving, ptr_t w, ptr_t bias, ptr_t labels,
                            std::vector<int> shape, float grad_scale, std::vector<ptr_t> out) {
  if (bn.size() != 9 || shape.size() != 5 || out.size() != 5)
    throw std::invalid_argument("head_fused: bn needs 9 pointers, shape 5 ints, out 5 pointers");
  HeadArgs a{};
  a.x = P<const bf16>(x);
  a.acc = P<const double>(bn[0]);
  a.gamma = P<const float>(bn[1]);
  a.beta = P<const float>(bn[2]);
  a.mmean = P<float>(bn[3]);
  a.mvar = P<float>(bn[4]);
  a.mean = P<float>(bn[5]);
  a.rstd = P<float>(bn[6]);
  a.scale = P<float>(bn[7]);
  a.shift = P<float>(bn[8]);
  a.momentum = momentum;
  a.eps = eps;
  a.update_moving = update_moving;
  a.w = P<const bf16>(w);
  a.bias = P<const float>(bias);
  a.labels = P<const int>(labels);
  a.N = shape[0];
  a.HW = shape[1];
  a.C = shape[2];
  a.classes = shape[3];
  a.kpad = shape[4];
  a.grad_scale = grad_scale;
  a.pooled = P<bf16>(out[0]);
  a.dlogits = P<bf16>(out[1]);
  a.ws = P<float>(out[2]);
  a.dact = P<bf16>(out[3]);
  a.bacc = P<double>(out[4]);
  if (!head_fused_supported(a.N, a.HW, a.C, a.classes, a.kpad))
    throw std::invalid_argument("head_fused: unsupported head shape");
  return [a](hipStream_t s) { head_fused(a, s); };
}

// Persistent small-batch CIFAR step (cifar_persist.hip).  mode 0: forward launch, 1:
// backward launch.  ptrs = [blocks, bns, x_in, stem_w, pool_acc, bar, err, dense_w,
// dense_b, labels, pooled, dlogits, ws, dpool, dx0, items]; ints = [nblocks, nitems, N, P,
// classes, kpad, update_moving, wgrad_wgs, fault_bar, overlap, bucket of stage 0, 1, 2];
// floats = [grad_scale, momentum, eps].
static Launch mk_prn(int mode, std::vector<ptr_t> p, std::vector<int> n, std::vector<float> f) {
  if (p.size() != 20 || n.size() != 13 || f.size() != 3)
    throw std::invalid_argument("prn: 20 pointers, 13 ints, 3 floats");
  PrnArgs a{};
  a.blocks = P<const PrnBlock>(p[0]);
  a.bns = P<const PrnBn>(p[1]);
  a.x_in = P<const bf16>(p[2]);
  a.stem_w = P<const bf16>(p[3]);
  a.pool_acc = P<double>(p[4]);
  a.bar = P<unsigned>(p[5]);
  a.err = P<int>(p[6]);
  a.dense_w = P<const bf16>(p[7]);
  a.dense_b = P<const float>(p[8]);
  a.labels = P<const int>(p[9]);
  a.pooled = P<bf16>(p[10]);
  a.dlogits = P<bf16>(p[11]);
  a.ws = P<float>(p[12]);
  a.dpool = P<float>(p[13]);
  a.dx0 = P<bf16>(p[14]);
  a.items = P<const PrnItem>(p[15]);
  a.loss_sum = P<float>(p[16]);
  a.correct = P<float>(p[17]);
  a.dbias = P<float>(p[18]);
  a.dense_grad = P<float>(p[19]);
  a.nblocks = n[0];
  a.nitems = n[1];
  a.N = n[2];
  a.P = n[3];
  a.classes = n[4];
  a.kpad = n[5];
  a.update_moving = n[6];
  const int wgs = n[7];
  a.fault_bar = n[8];
  a.overlap = n[9];
  for (int i = 0; i < 3; ++i) a.bucket_of_stage[i] = n[10 + i];
  a.grad_scale = f[0];
  a.momentum = f[1];
  a.eps = f[2];
  if (!prn_supported(a.N, a.P, a.nblocks, a.classes, a.kpad))
    throw std::invalid_argument("prn: unsupported shape");
  if (mode == 0) return [a](hipStream_t s) { prn_forward(a, s); };
  if (mode == 1) return [a, wgs](hipStream_t s) { prn_backward(a, wgs, s); };
  if (mode == 2) return [a](hipStream_t s) { prn_head(a, s); };
  throw std::invalid_argument("prn: mode 0 (forward), 1 (backward) or 2 (head folds)");
}

static Launch mk_prn_bucket_wait(ptr_t bar, int bucket, long long target, ptr_t err) {
  return [=](hipStream_t s) { prn_bucket_wait(P<unsigned>(bar), bucket, (unsigned)target, P<int>(err), s); };
}

// bn_bwd_apply with the finalize fused in: fin = [acc, gamma, dgamma, dbeta, coef]
static Launch mk_bn_bwd_apply_acc(ptr_t dy, ptr_t x, ptr_t mean, ptr_t rstd, ptr_t scale,
                                  ptr_t shift, std::vector<ptr_t> fin, ptr_t add, ptr_t dx, int M,
                                  int C) {
  if (fin.size() != 5) throw std::invalid_argument("bn_bwd_apply_acc: fin needs 5 pointers");
  if (!bn_bwd_apply_acc_fits(M, C))
    throw std::invalid_argument("bn_bwd_apply_acc: shape exceeds the fused-finalize bound");
  const BwdAccFin f{P<const double>(fin[0]), P<const float>(fin[1]), P<float>(fin[2]),
                    P<float>(fin[3]), P<float>(fin[4]), M};
  return [=](hipStream_t s) {
    bn_relu_bwd_apply_acc(P<const bf16>(dy), P<const bf16>(x), P<const float>(mean),
                          P<const float>(rstd), P<const float>(scale), P<const float>(shift), f,
                          P<const bf16>(add), P<bf16>(dx), M, C, s);
  };
}

static Launch mk_maxpool_fwd(ptr_t x, ptr_t y, ptr_t argmax, std::vector<int> geom, int k) {
  ConvGeom g = geom_from(geom);
  if (g.C % 8) throw std::invalid_argument("maxpool: C % 8");
  return [=](hipStream_t s) {
    maxpool_fwd(P<const bf16>(x), P<bf16>(y), P<uint8_t>(argmax), g.N, g.H, g.W, g.C, g.Ho, g.Wo,
                k, g.stride, g.pad, s);
  };
}

static Launch mk_maxpool_bwd(ptr_t argmax, ptr_t dy, ptr_t dx, std::vector<int> geom, int k) {
  ConvGeom g = geom_from(geom);
  if (g.C % 8) throw std::invalid_argument("maxpool: C % 8");
  return [=](hipStream_t s) {
    maxpool_bwd(P<const uint8_t>(argmax), P<const bf16>(dy), P<bf16>(dx), g.N, g.H, g.W, g.C, g.Ho,
                g.Wo, k, g.stride, g.pad, s);
  };
}

static LrSchedule make_sched(float init, long long warm_steps, float warm_from, float warm_to,
                             std::vector<long long> bounds, std::vector<float> vals) {
  LrSchedule sc{};
  if (bounds.size() > 7 || vals.size() != bounds.size() + 1)
    throw std::invalid_argument("lr schedule: <=7 bounds and len(vals)==len(bounds)+1");
  sc.init = init;
  sc.warm_steps = warm_steps;
  sc.warm_from = warm_from;
  sc.warm_to = warm_to;
  sc.nb = (int)bounds.size();
  for (size_t i = 0; i < bounds.size(); ++i) sc.bound[i] = bounds[i];
  for (size_t i = 0; i < vals.size(); ++i) sc.val[i] = vals[i];
  return sc;
}

static Launch mk_ohwi_pack(ptr_t master, ptr_t segs, ptr_t tile0, int nseg, long long tiles,
                           ptr_t bf, ptr_t gstep_inc) {
  return [=](hipStream_t s) {
    ohwi_pack(P<const float>(master), P<const ParamSeg>(segs), P<const long long>(tile0), nseg,
              tiles, P<bf16>(bf), P<long long>(gstep_inc), s);
  };
}

static Launch mk_sgd_update_pack(ptr_t master, ptr_t grad, ptr_t mom, long n, float init,
                                 long long warm_steps, float warm_from, float warm_to,
                                 std::vector<long long> bounds, std::vector<float> vals,
                                 ptr_t gstep, float momentum, float wd, float grad_scale,
                                 int use_momentum, ptr_t segs, int nseg, ptr_t bf, ptr_t lr_out,
                                 int update) {
  const LrSchedule sc = make_sched(init, warm_steps, warm_from, warm_to, bounds, vals);
  return [=](hipStream_t s) {
    sgd_update_pack(P<float>(master), P<const float>(grad), P<float>(mom), n, sc,
                    P<const long long>(gstep), momentum, wd, grad_scale, use_momentum,
                    P<const ParamSeg>(segs), nseg, P<bf16>(bf), P<float>(lr_out), update, s);
  };
}

static Launch mk_sgd_tiles(ptr_t master, ptr_t grad, ptr_t mom, float init,
                           long long warm_steps, float warm_from, float warm_to,
                           std::vector<long long> bounds, std::vector<float> vals, ptr_t gstep,
                           float momentum, float wd, float grad_scale, int use_momentum,
                           ptr_t segs, ptr_t work, ptr_t blk_seg, int nblocks, ptr_t bf,
                           ptr_t lr_out, ptr_t ticket, ptr_t gin, ptr_t gout, int pack) {
  const LrSchedule sc = make_sched(init, warm_steps, warm_from, warm_to, bounds, vals);
  return [=](hipStream_t s) {
    sgd_tiles(P<float>(master), P<float>(grad), P<float>(mom), sc, P<long long>(gstep),
              momentum, wd, grad_scale, use_momentum, P<const ParamSeg>(segs),
              P<const OptWork>(work), P<const int>(blk_seg), nblocks, P<bf16>(bf),
              P<float>(lr_out), P<unsigned>(ticket), P<const bf16>(gin), P<bf16>(gout), pack, s);
  };
}

static Launch mk_step_increment(ptr_t gstep) {
  return [=](hipStream_t s) { step_increment(P<long long>(gstep), s); };
}

static Launch mk_l2_half_sum(ptr_t v, long n, ptr_t ws, ptr_t out) {
  return [=](hipStream_t s) { l2_half_sum(P<const float>(v), n, P<float>(ws), P<float>(out), s); };
}

static Launch mk_fill(ptr_t p, long n, float a) {
  return [=](hipStream_t s) { fill_f32(P<float>(p), n, a, s); };
}

static Launch mk_delay(double us) {   // diagnostics: one spinning wave (diag.hip)
  const long long ticks = (long long)(us * 100.0);
  return [=](hipStream_t s) { plan_delay(ticks, s); };
}

static Launch mk_memset(ptr_t p, long bytes) {
  return [=](hipStream_t s) {
    if (hipMemsetAsync(P<void>(p), 0, (size_t)bytes, s) != hipSuccess)
      fprintf(stderr, "hipMemsetAsync failed\n");
  };
}

static Launch mk_cifar_augment(ptr_t img, ptr_t out, int N, int H, int W, int Cpad, int pad,
                               unsigned long long seed, ptr_t gstep, int train, ptr_t crop_log,
                               ptr_t zero, long zero_bytes) {
  if (zero_bytes % 16) throw std::invalid_argument("cifar_augment: zero_bytes % 16 != 0");
  return [=](hipStream_t s) {
    cifar_augment(P<const uint8_t>(img), P<bf16>(out), N, H, W, Cpad, pad, seed,
                  P<const long long>(gstep), train, P<int>(crop_log), P<void>(zero), zero_bytes,
                  s);
  };
}

static Launch mk_imagenet_u8_pack(ptr_t img, ptr_t out, int N, int H, int W,
                                  unsigned long long seed, ptr_t gstep, int train, ptr_t zero,
                                  long zero_bytes, int s2d) {
  if (zero_bytes % 16) throw std::invalid_argument("imagenet_u8_pack: zero_bytes % 16 != 0");
  if (s2d && ((H | W) & 1)) throw std::invalid_argument("imagenet_u8_pack: s2d needs even H, W");
  return [=](hipStream_t s) {
    imagenet_u8_pack(P<const uint8_t>(img), P<bf16>(out), N, H, W, seed,
                     P<const long long>(gstep), train, P<void>(zero), zero_bytes, s2d, s);
  };
}

static Launch mk_stem_s2d_pack(ptr_t w7, ptr_t w4, int K) {
  return [=](hipStream_t s) { stem_s2d_pack(P<const float>(w7), P<bf16>(w4), K, s); };
}

static Launch mk_stem_s2d_grad(ptr_t g4, ptr_t g7, int K) {
  return [=](hipStream_t s) { stem_s2d_grad(P<const float>(g4), P<float>(g7), K, s); };
}

static Launch mk_pad_channels(ptr_t x, ptr_t out, long npix, int C, int Cpad) {
  return [=](hipStream_t s) { nhwc_pad_channels(P<const float>(x), P<bf16>(out), npix, C, Cpad, s); };
}

static Launch mk_synthetic(ptr_t out, long npix, int C, int Cpad, unsigned long long seed) {
  return [=](hipStream_t s) { synthetic_images(P<bf16>(out), npix, C, Cpad, seed, s); };
}

static Launch mk_cast_f2b(ptr_t a, ptr_t b, long n) {
  return [=](hipStream_t s) { cast_f32_bf16(P<const float>(a), P<bf16>(b), n, s); };
}
static Launch mk_cast_b2f(ptr_t a, ptr_t b, long n) {
  return [=](hipStream_t s) { cast_bf16_f32(P<const bf16>(a), P<float>(b), n, s); };
}

// ---------------------------------------------------------------- Plan
// A plan is a list of ops, each bound to one of three streams (0 = main
// compute, 1 = side compute for weight gradients, 2 = RCCL comm), plus
// cross-stream event record/wait ops.  Recording a stream's first op behind a
// wait on another stream's event makes the fork/join structure explicit (and
// capturable into a hipGraph: the waits become graph edges).  The structure is
// checked host-side when a plan is built (utils/streamcheck.py).
enum OpKind { OP_LAUNCH = 0, OP_RECORD = 1, OP_WAIT = 2, OP_TIMING = 3 };
constexpr int PLAN_STREAMS = 3;

struct PlanOp {
  Launch fn;       // launch (OP_LAUNCH)
  int stream;      // 0 main, 1 side, 2 comm
  int kind;        // OpKind
  int ev;          // event index (record / wait), timing-event index (OP_TIMING)
};

// One host thread per stream (Plan::run, threaded mode).  hipLaunchKernel costs
// ~3 us of host time; issued from one thread, the side stream's weight-gradient
// launches sit between the main stream's dgrad launches, and at small batch
// (CIFAR, 16-32 images per rank) the main stream drains while the host is busy
// with the side stream (rocprofv3 timeline: ~35 us main-stream gaps every two
// residual blocks).  Each stream's ops are instead issued, in plan order, by its
// own thread; a cross-stream wait is issued only once the matching record has
// been issued in THIS run (per-op generation stamps), so the device-side
// fork/join graph is exactly the single-threaded one.
struct IssueWorker {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::function<void()> job;
  bool has_job = false, quit = false, done = true;
  IssueWorker() {
    th = std::thread([this] {
      for (;;) {
        std::function<void()> j;
        {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [this] { return has_job || quit; });
          if (quit) return;
          j = std::move(job);
          has_job = false;
        }
        j();
        {
          std::lock_guard<std::mutex> lk(mu);
          done = true;
        }
        cv.notify_all();
      }
    });
  }
  void start(std::function<void()> j) {
    {
      std::lock_guard<std::mutex> lk(mu);
      job = std::move(j);
      has_job = true;
      done = false;
    }
    cv.notify_all();
  }
  void join() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [this] { return done; });
  }
  ~IssueWorker() {
    {
      std::lock_guard<std::mutex> lk(mu);
      quit = true;
    }
    cv.notify_all();
    if (th.joinable()) th.join();
  }
};

struct Plan {
  std::vector<PlanOp> ops;
  std::unique_ptr<PlanSplitK> splitk[3];   // per stream (PLAN_STREAMS)
  PlanSplitK* splitk_ws(int stream) {
    if (!splitk[stream]) splitk[stream].reset(new PlanSplitK());
    return splitk[stream].get();
  }
  std::vector<std::string> names;
  std::vector<hipEvent_t> events;
  std::vector<hipEvent_t> tevents;            // timing events (OP_TIMING)
  std::vector<std::shared_ptr<void>> keep;   // objects the launches reference (communicators)
  std::vector<double> host_us;   // per-op host issue time (profile mode only)
  bool profile = false;
  bool timing = false;           // OP_TIMING ops record only when enabled
  int threaded = -1;             // -1: DTR_PLAN_THREADS (default 1); 0 / 1
  int cur = 0;
  // threaded issue state
  std::unique_ptr<IssueWorker> workers[PLAN_STREAMS];
  std::unique_ptr<std::atomic<unsigned>[]> stamp;   // generation at which op i was issued
  size_t stamp_n = 0;
  std::vector<int> rec_of;       // WAIT op -> latest RECORD op of its event before it (-1)
  size_t rec_of_n = 0;
  unsigned gen = 0;
  std::atomic<bool> abort_run{false};
  std::mutex err_mu;
  std::string err_msg;           // first exception message of a threaded run
  // schedule perturbation (race check, utils/racecheck.py): 0 off; 1 serialize every
  // stream onto the main stream (plan order = a valid sequential schedule); 2 jitter:
  // a plan_delay of U[0, pmax_ticks) in front of a launch with probability pprob,
  // drawn from (pseed, run, op) so each run perturbs a different schedule
  int perturb = 0;
  unsigned long long pseed = 0, prun = 0;
  double pprob = 0.0;
  long long pmax_ticks = 0;

  static unsigned long long mix64(unsigned long long x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
  }
  void set_perturb(int mode, unsigned long long seed, double prob, double max_us) {
    if (mode < 0 || mode > 2) throw std::invalid_argument("perturb mode: 0 off, 1 serialize, 2 jitter");
    perturb = mode;
    pseed = seed;
    prun = 0;
    pprob = prob;
    pmax_ticks = (long long)(max_us * 100.0);   // wall clock: 100 MHz
  }

  ~Plan() {
    for (auto& w : workers) w.reset();
    for (auto e : events) (void)hipEventDestroy(e);
    for (auto e : tevents) (void)hipEventDestroy(e);
  }
  int add(Launch l, const std::string& name) {
    ops.push_back(PlanOp{std::move(l), cur, OP_LAUNCH, -1});
    names.push_back(name);
    return (int)ops.size() - 1;
  }
  int new_event() {
    // Plan events only order streams of this device (the comm stream's collective kernels
    // run here too), and every producing kernel's own end-of-kernel release already makes
    // its writes visible device-wide: the record's marker needs no fence of its own.  tune
    // plan_event_scope: 2 (default) no marker fence -- CIFAR RN50 bs128 1.305 -> 1.280 ms,
    // bs16 0.951 -> 0.932 (scripts/gpu_r3_events.sh; ImageNet within noise) -- 1 device-
    // scope release (measured = 0), 0 the runtime default (system-scope release).
    const long scope = tune(T_PLAN_EVENT_SCOPE);
    unsigned flags = hipEventDisableTiming;
    if (scope == 1) flags |= hipEventReleaseToDevice;
    if (scope == 2) flags |= hipEventDisableSystemFence;
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, flags) != hipSuccess)
      throw std::runtime_error("hipEventCreate failed");
    events.push_back(e);
    return (int)events.size() - 1;
  }
  int record(int ev) {
    if (ev < 0 || ev >= (int)events.size()) throw std::out_of_range("record: unknown event");
    ops.push_back(PlanOp{Launch(), cur, OP_RECORD, ev});
    names.push_back("record");
    return (int)ops.size() - 1;
  }
  int wait(int ev) {
    if (ev < 0 || ev >= (int)events.size()) throw std::out_of_range("wait: unknown event");
    ops.push_back(PlanOp{Launch(), cur, OP_WAIT, ev});
    names.push_back("wait");
    return (int)ops.size() - 1;
  }
  // A timing probe on the current stream (HIP event with timing); a no-op unless
  // set_timing(true).  Not a synchronisation op: the stream check ignores it.
  int timing_point(const std::string& label) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) throw std::runtime_error("hipEventCreate failed");
    tevents.push_back(e);
    ops.push_back(PlanOp{Launch(), cur, OP_TIMING, (int)tevents.size() - 1});
    names.push_back("timing:" + label);
    return (int)ops.size() - 1;
  }
  double elapsed_ms(int op_a, int op_b) const {
    for (int i : {op_a, op_b})
      if (i < 0 || i >= (int)ops.size() || ops[i].kind != OP_TIMING)
        throw std::invalid_argument("elapsed_ms: not a timing op");
    float ms = 0.f;
    const hipError_t e = hipEventElapsedTime(&ms, tevents[ops[op_a].ev], tevents[ops[op_b].ev]);
    if (e != hipSuccess)
      throw std::runtime_error(std::string("hipEventElapsedTime: ") + hipGetErrorString(e));
    return ms;
  }

  hipError_t issue(int i, hipStream_t s) {
    const PlanOp& o = ops[i];
    if (o.kind == OP_LAUNCH) {
      if (perturb == 2 && pmax_ticks > 0) {
        const unsigned long long h = mix64(mix64(pseed ^ (prun << 32)) ^ (unsigned long long)i);
        if ((double)(h >> 11) * (1.0 / 9007199254740992.0) < pprob)
          plan_delay((long long)(mix64(h) % (unsigned long long)pmax_ticks), s);
      }
      o.fn(s);
      return hipSuccess;
    }
    if (o.kind == OP_RECORD) return hipEventRecord(events[o.ev], s);
    if (o.kind == OP_WAIT) return hipStreamWaitEvent(s, events[o.ev], 0);
    if (timing) return hipEventRecord(tevents[o.ev], s);
    return hipSuccess;
  }

  bool use_threads(int begin, int end) {
    if (threaded < 0) {
      const char* e = std::getenv("DTR_PLAN_THREADS");
      threaded = (e != nullptr && e[0] == '0') ? 0 : 1;
    }
    if (!threaded || profile) return false;
    bool multi = false;
    for (int i = begin; i < end && !multi; ++i) multi = ops[i].stream != ops[begin].stream;
    return multi;
  }

  void prepare_threads() {
    if (stamp_n != ops.size()) {
      stamp.reset(new std::atomic<unsigned>[ops.size()]);
      for (size_t i = 0; i < ops.size(); ++i) stamp[i].store(0u);
      stamp_n = ops.size();
    }
    if (rec_of_n != ops.size()) {
      rec_of.assign(ops.size(), -1);
      std::vector<int> last(events.size(), -1);
      for (size_t i = 0; i < ops.size(); ++i) {
        if (ops[i].kind == OP_RECORD) last[ops[i].ev] = (int)i;
        else if (ops[i].kind == OP_WAIT) rec_of[i] = last[ops[i].ev];
      }
      rec_of_n = ops.size();
    }
    for (int s = 1; s < PLAN_STREAMS; ++s)
      if (!workers[s]) workers[s].reset(new IssueWorker());
  }

  // Issue stream `sid`'s ops of [begin, end) in order; returns the first failure.
  std::pair<int, hipError_t> issue_stream(int sid, int begin, int end, hipStream_t s, unsigned g) {
    if (sid != 0) {   // the current device is per host thread: use the stream's
      int dev = -1, curdev = -1;
      if (hipStreamGetDevice(s, &dev) == hipSuccess && hipGetDevice(&curdev) == hipSuccess &&
          dev >= 0 && dev != curdev)
        (void)hipSetDevice(dev);
    }
    for (int i = begin; i < end; ++i) {
      if (ops[i].stream != sid) continue;
      if (ops[i].kind == OP_WAIT) {
        const int r = rec_of[i];
        if (r >= begin) {   // recorded in this range: wait until it is issued in this run
          unsigned spins = 0;
          while (stamp[r].load(std::memory_order_acquire) != g) {
            if (abort_run.load(std::memory_order_relaxed)) return {i, hipErrorUnknown};
            if (++spins > 64) std::this_thread::yield();
          }
        }
      }
      hipError_t e = hipSuccess;
      try {   // a launch closure may throw (shape / coverage checks): never out of a thread
        e = issue(i, s);
      } catch (const std::exception& ex) {
        std::lock_guard<std::mutex> lk(err_mu);
        if (err_msg.empty()) err_msg = ex.what();
        e = hipErrorInvalidValue;
      }
      if (e == hipSuccess && ops[i].kind == OP_LAUNCH) e = hipGetLastError();  // per thread
      if (e != hipSuccess) {
        abort_run.store(true);
        return {i, e};
      }
      stamp[i].store(g, std::memory_order_release);
    }
    return {-1, hipSuccess};
  }

  void run(int begin, int end, ptr_t main_stream, ptr_t side_stream, ptr_t comm_stream) {
    if (begin < 0 || end > (int)ops.size() || begin > end) throw std::out_of_range("plan range");
    hipStream_t st[PLAN_STREAMS] = {S(main_stream), S(side_stream ? side_stream : main_stream),
                                    S(comm_stream ? comm_stream : main_stream)};
    if (perturb == 1) st[1] = st[2] = st[0];   // sequential: plan order on one stream
    ++prun;
    int bad_op = -1;
    hipError_t bad = hipSuccess;
    // Never while capturing a hipGraph: capture from several host threads is not
    // reliable on this runtime (capture_end failed with hipErrorInvalidValue in one
    // of three runs); the graph replays without host issue cost anyway.
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(st[0], &cap);
    if (cap == hipStreamCaptureStatusNone && use_threads(begin, end) && st[1] != st[0] &&
        st[2] != st[0] && st[1] != st[2]) {
      py::gil_scoped_release nogil;
      prepare_threads();
      const unsigned g = ++gen == 0 ? ++gen : gen;   // 0 = never issued
      abort_run.store(false);
      err_msg.clear();
      std::pair<int, hipError_t> res[PLAN_STREAMS];
      bool used[PLAN_STREAMS] = {false, false, false};
      for (int i = begin; i < end; ++i) used[ops[i].stream] = true;
      for (int sid = 1; sid < PLAN_STREAMS; ++sid) {
        res[sid] = {-1, hipSuccess};
        if (used[sid])
          workers[sid]->start([this, sid, begin, end, &st, g, &res] {
            res[sid] = issue_stream(sid, begin, end, st[sid], g);
          });
      }
      res[0] = issue_stream(0, begin, end, st[0], g);
      for (int sid = 1; sid < PLAN_STREAMS; ++sid)
        if (used[sid]) workers[sid]->join();
      for (auto& r : res)
        if (r.second != hipSuccess && (bad_op < 0 || r.first < bad_op)) {
          bad_op = r.first;
          bad = r.second;
        }
    } else {
      py::gil_scoped_release nogil;
      if (profile && host_us.size() != ops.size()) host_us.assign(ops.size(), 0.0);
      for (int i = begin; i < end; ++i) {
        const auto t0 = profile ? std::chrono::steady_clock::now()
                                : std::chrono::steady_clock::time_point();
        // A failed record/wait silently drops a fork or join the stream check
        // certified: remember the first failure and stop issuing.
        const hipError_t e = issue(i, st[ops[i].stream]);
        if (e != hipSuccess) {
          bad_op = i;
          bad = e;
          break;
        }
        if (profile)
          host_us[i] += std::chrono::duration<double, std::micro>(
                            std::chrono::steady_clock::now() - t0).count();
      }
      if (bad == hipSuccess) {
        const hipError_t e = hipGetLastError();   // a failed kernel launch anywhere in the range
        if (e != hipSuccess) {
          bad = e;
          bad_op = end - 1;
        }
      }
    }
    if (bad != hipSuccess)
      throw std::runtime_error("plan op " + std::to_string(bad_op) + " (" + names[bad_op] +
                               ") failed: " + (err_msg.empty() ? hipGetErrorString(bad)
                                                               : err_msg.c_str()));
  }
  int size() const { return (int)ops.size(); }
};

// Register `name` both as an immediate op (trailing stream arg) and as a Plan
// recorder (returns the op index).
template <typename R, typename... Args>
static void def_op(py::module_& m, py::class_<Plan>& plan, const char* name,
                   R (*maker)(Args...)) {
  m.def(name, [maker, name](Args... args, ptr_t stream) {
    maker(args...)(S(stream));
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess)
      throw std::runtime_error(std::string(name) + " launch failed: " + hipGetErrorString(e));
  });
  plan.def(name, [maker, name](Plan& p, Args... args) {
    g_rec_splitk = p.splitk_ws(p.cur);
    Launch l;
    try {
      l = maker(args...);
    } catch (...) {
      g_rec_splitk = nullptr;
      throw;
    }
    g_rec_splitk = nullptr;
    return p.add(std::move(l), name);
  });
}

namespace dtr {
uint32_t crc32c_extend(uint32_t crc, const uint8_t* p, size_t n);
}

static int hip_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "gfx950 (MI355X) native kernels + static-plan executor for ResNet training";
  py::class_<Plan> plan(m, "Plan");
  plan.def(py::init<>())
      .def("run", &Plan::run, py::arg("begin"), py::arg("end"), py::arg("stream"),
           py::arg("side_stream") = 0, py::arg("comm_stream") = 0)
      .def("size", &Plan::size)
      .def("set_perturb", &Plan::set_perturb, py::arg("mode"), py::arg("seed") = 0,
           py::arg("prob") = 0.0, py::arg("max_us") = 0.0)
      .def("new_event", &Plan::new_event)
      .def("record", &Plan::record)
      .def("wait", &Plan::wait)
      .def("use_stream", [](Plan& p, int s) {
        if (s < 0 || s >= PLAN_STREAMS)
          throw std::invalid_argument("stream index must be 0 (main), 1 (side) or 2 (comm)");
        p.cur = s;
      })
      .def("current_stream", [](const Plan& p) { return p.cur; })
      .def("timing_point", &Plan::timing_point)
      .def("set_timing", [](Plan& p, bool on) { p.timing = on; })
      .def("set_threaded", [](Plan& p, bool on) { p.threaded = on ? 1 : 0; })
      .def("elapsed_ms", &Plan::elapsed_ms)
      // in-place SUM all-reduce of `count` elements at `ptr` on the plan's current
      // stream through the native communicator (dtype: 7 fp32, 9 bf16; any transport)
      .def("all_reduce", [](Plan& p, std::shared_ptr<Comm> c, ptr_t ptr, long long count,
                            int dtype) {
        if (!c) throw std::invalid_argument("all_reduce: no communicator");
        if (count <= 0) throw std::invalid_argument("all_reduce: empty buffer");
        Comm* cp = c.get();
        p.keep.push_back(c);
        return p.add([cp, ptr, count, dtype](hipStream_t s) {
          cp->all_reduce(P<void>(ptr), (size_t)count, dtype, s);
        }, "all_reduce");
      })
      .def("names", [](const Plan& p) { return p.names; })
      .def("set_profile", [](Plan& p, bool on) {
        p.profile = on;
        if (on) p.host_us.clear();
      })
      .def("host_us", [](const Plan& p) { return p.host_us; })
      .def("op_streams", [](const Plan& p) {
        std::vector<int> v;
        for (const auto& o : p.ops) v.push_back(o.stream);
        return v;
      })
      // (kind, event) per op for the host-side stream-ordering check
      // (utils/streamcheck.py): kind 0 launch, 1 record, 2 wait; event -1 for launches.
      .def("op_kinds", [](const Plan& p) {
        std::vector<int> v;
        for (const auto& o : p.ops) v.push_back(o.kind);
        return v;
      })
      .def("op_events", [](const Plan& p) {
        std::vector<int> v;
        for (const auto& o : p.ops) v.push_back(o.ev);
        return v;
      });

  // Native communicator (comm.h).  Construction is collective and blocks until
  // every rank has joined, and a host-staged (shm) collective blocks its caller,
  // so the GIL is released around both.
  py::class_<Comm, std::shared_ptr<Comm>>(m, "Comm")
      .def(py::init([](py::bytes id, int world, int rank, int device) {
             std::string uid = id;
             py::gil_scoped_release nogil;
             return std::make_shared<Comm>(uid, world, rank, device);
           }),
           py::arg("unique_id"), py::arg("world"), py::arg("rank"), py::arg("device"))
      .def_static("shm", [](const std::string& name, int world, int rank, int device,
                            long long slot_bytes, double timeout_s, double init_timeout_s) {
             py::gil_scoped_release nogil;
             return std::shared_ptr<Comm>(Comm::shm(name, world, rank, device, (size_t)slot_bytes,
                                                    timeout_s, init_timeout_s));
           },
           py::arg("name"), py::arg("world"), py::arg("rank"), py::arg("device"),
           py::arg("slot_bytes") = 64ll << 20, py::arg("timeout_s") = 600.0,
           py::arg("init_timeout_s") = 0.0)
      .def_static("loopback", [](float factor) { return std::shared_ptr<Comm>(Comm::loopback(factor)); },
                  py::arg("factor") = 2.0f)
      .def("all_reduce", [](Comm& c, ptr_t p, long long n, int dtype, ptr_t s) {
        py::gil_scoped_release nogil;
        c.all_reduce(P<void>(p), (size_t)n, dtype, S(s));
      })
      .def("broadcast", [](Comm& c, ptr_t p, long long n, int dtype, int root, ptr_t s) {
        py::gil_scoped_release nogil;
        c.broadcast(P<void>(p), (size_t)n, dtype, root, S(s));
      })
      .def("host_all_reduce", [](Comm& c, ptr_t p, long long n, int dtype) {
        py::gil_scoped_release nogil;
        c.host_all_reduce(P<void>(p), (size_t)n, dtype);
      })
      .def("host_broadcast", [](Comm& c, ptr_t p, long long n, int dtype, int root) {
        py::gil_scoped_release nogil;
        c.host_broadcast(P<void>(p), (size_t)n, dtype, root);
      })
      .def("async_error", &Comm::async_error)
      .def("abort", &Comm::abort)
      .def_property_readonly("world", &Comm::world)
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("transport", &Comm::transport)
      .def_property_readonly("library_path", &Comm::library_path)
      .def_static("unique_id", []() { return py::bytes(Comm::unique_id()); })
      .def_static("library", &Comm::library)
      .def_static("rccl_available", &Comm::rccl_available)
      .def_static("rccl_version", &Comm::rccl_version);
  m.attr("COMM_F32") = (int)COMM_F32;
  m.attr("COMM_BF16") = (int)COMM_BF16;
  m.attr("COMM_F64") = (int)COMM_F64;
  m.attr("COMM_I64") = (int)COMM_I64;

  def_op(m, plan, "conv_gemm", mk_conv_gemm);
  def_op(m, plan, "conv_wgrad", mk_conv_wgrad);
  def_op(m, plan, "wgrad_reduce", mk_wgrad_reduce);
  def_op(m, plan, "wgrad_reduce_grouped", mk_wgrad_reduce_grouped);
  def_op(m, plan, "bn_finalize", mk_bn_finalize);
  def_op(m, plan, "bn_eval", mk_bn_eval);
  def_op(m, plan, "bn_stats", mk_bn_stats);
  def_op(m, plan, "bn_bwd_reduce", mk_bn_bwd_reduce);
  def_op(m, plan, "bn_bwd_finalize", mk_bn_bwd_finalize);
  def_op(m, plan, "bnd1x1", mk_bnd1x1);
  def_op(m, plan, "bnf1x1", mk_bnf1x1);
  m.def("bnf1x1_covers", &bnf1x1_covers, "whether the streaming narrow-K 1x1 forward (+ BN prologue, residual, BN statistics) covers (M, C, K)");
  m.def("bnd1x1_covers", &bnd1x1_covers, "whether the streaming narrow-K 1x1 dgrad + BN backward covers (M, C, K)");
  def_op(m, plan, "bn_bwd_apply", mk_bn_bwd_apply);
  def_op(m, plan, "bn_relu_apply", mk_bn_relu_apply);
  def_op(m, plan, "bn_relu_apply_acc", mk_bn_relu_apply_acc);
  def_op(m, plan, "bnrelu_avgpool", mk_bnrelu_avgpool);
  def_op(m, plan, "avgpool_bwd", mk_avgpool_bwd);
  def_op(m, plan, "softmax_xent", mk_softmax_xent);
  def_op(m, plan, "softmax_xent_reduce", mk_softmax_xent_reduce);
  def_op(m, plan, "bn_bwd_apply_acc", mk_bn_bwd_apply_acc);
  m.def("bn_bwd_apply_acc_fits", &bn_bwd_apply_acc_fits,
        "whether bn_bwd_apply_acc (finalize fused into the apply) covers (M, C)");
  def_op(m, plan, "head_fused", mk_head_fused);
  def_op(m, plan, "prn", mk_prn);
  def_op(m, plan, "prn_bucket_wait", mk_prn_bucket_wait);
  m.def("prn_set_probe", [](ptr_t p) { prn_set_probe(P<long long>(p)); },
        "diagnostics: image 0 of the persistent launches records (tag, wall clock) pairs here");
  m.def("prn_supported", &prn_supported, "whether the persistent CIFAR step covers (N, slices, blocks, classes, kpad)");
  m.def("prn_check", &prn_check, "every host-side limit of the persistent step (N, slices, forward slices, "
        "blocks, classes, kpad), co-residency included: '' or the reason it is unsupported");
  m.def("prn_item_kind", &prn_item_kind, "weight-gradient item kind of a conv (cin, cout, k, stride)");
  m.def("prn_struct_bytes", []() {
    return std::vector<int>{(int)sizeof(PrnBn), (int)sizeof(PrnBlock), (int)sizeof(PrnItem)};
  }, "sizeof PrnBn, PrnBlock, PrnItem (descriptor tables built in Python)");
  m.def("head_fused_supported", &head_fused_supported,
        "whether head_fused covers (N, HW, C, classes, kpad)");
  def_op(m, plan, "maxpool_fwd", mk_maxpool_fwd);
  def_op(m, plan, "maxpool_bwd", mk_maxpool_bwd);
  def_op(m, plan, "sgd_update_pack", mk_sgd_update_pack);
  def_op(m, plan, "ohwi_pack", mk_ohwi_pack);
  def_op(m, plan, "sgd_tiles", mk_sgd_tiles);
  def_op(m, plan, "step_increment", mk_step_increment);
  def_op(m, plan, "l2_half_sum", mk_l2_half_sum);
  def_op(m, plan, "fill", mk_fill);
  def_op(m, plan, "memset", mk_memset);
  def_op(m, plan, "delay", mk_delay);
  def_op(m, plan, "cifar_augment", mk_cifar_augment);
  def_op(m, plan, "imagenet_u8_pack", mk_imagenet_u8_pack);
  def_op(m, plan, "stem_s2d_pack", mk_stem_s2d_pack);
  def_op(m, plan, "stem_s2d_grad", mk_stem_s2d_grad);
  def_op(m, plan, "pad_channels", mk_pad_channels);
  def_op(m, plan, "synthetic_images", mk_synthetic);
  def_op(m, plan, "cast_f32_bf16", mk_cast_f2b);
  def_op(m, plan, "cast_bf16_f32", mk_cast_b2f);

  // host-side helpers that mirror the launchers' internal choices
  m.def("conv_gemm_bm", &conv_gemm_bm);
  m.def("conv_gemm_splitk_bytes", [](int mode, std::vector<int> geom) {
    GemmArgs g{};
    g.g = geom_from(geom);
    const ConvGeom& c = g.g;
    g.M = mode == MODE_FWD ? c.N * c.Ho * c.Wo : c.N * c.H * c.W;
    g.Ncol = mode == MODE_FWD ? c.K : c.C;
    g.Kdim = c.kh * c.kw * (mode == MODE_FWD ? c.C : c.K);
    size_t tiles = 0;
    return (long long)conv_gemm_splitk_need(g, mode, &tiles);
  }, "split-K slab bytes conv_gemm would use for a plain conv of this geometry (0: none)");
  m.def("conv_gemm_bn", &conv_gemm_bn);
  m.def("conv_direct_covers", [](int mode, std::vector<int> geom) {
    GemmArgs g{};
    g.g = geom_from(geom);
    const ConvGeom& c = g.g;
    g.M = mode == MODE_FWD ? c.N * c.Ho * c.Wo : c.N * c.H * c.W;
    g.Ncol = mode == MODE_FWD ? c.K : c.C;
    return conv_direct_covers(g, mode);
  }, "whether conv_gemm(mode, geom) runs the direct 3x3 kernel");
  m.def("conv_ring_covers", [](int mode, std::vector<int> geom) {
    GemmArgs g{};
    g.g = geom_from(geom);
    const ConvGeom& c = g.g;
    g.M = mode == MODE_FWD ? c.N * c.Ho * c.Wo : c.N * c.H * c.W;
    g.Ncol = mode == MODE_FWD ? c.K : c.C;
    g.Kdim = c.kh * c.kw * (mode == MODE_FWD ? c.C : c.K);
    return conv_gemm_uses_ring(g, mode);
  }, "whether conv_gemm(mode, geom) (no BN+ReLU prologue) runs the LDS-DMA ring loop");
  m.def("set_direct_probe", [](ptr_t p) { set_direct_probe(P<long long>(p)); },
        "diagnostics: direct-conv workgroups write 4 wall-clock stamps each to p (0 = off)");
  m.def("set_wgrad_direct", &set_wgrad_direct,
        "enable/disable the direct 3x3 small-C wgrad kernel (tune direct_wgrad); changes "
        "wgrad_pick_splits, so set it before planning");
  m.def("set_conv_direct", &set_conv_direct,
        "enable/disable the direct 3x3 small-C conv kernel (tune direct_conv)");
  m.def("set_conv_pipeline", &set_conv_pipeline,
        "enable/disable the 2-deep pipelined implicit-GEMM / wgrad loops (tune conv_pipe)");
  m.def("tune_table", []() {
    py::list out;
    const TuneEntry* t = tune_table();
    for (int i = 0; i < T_COUNT; ++i)
      out.append(py::make_tuple(t[i].key, t[i].dflt, t[i].doc, tune((TuneId)i)));
    return out;
  }, "(key, default, doc, current value) of every native tuning entry (csrc/tune.h)");
  m.def("tune_set", [](const std::string& key, long v) {
    const TuneEntry* t = tune_table();
    for (int i = 0; i < T_COUNT; ++i)
      if (key == t[i].key) {
        tune_set((TuneId)i, v);
        return;
      }
    throw std::invalid_argument("unknown native tuning key " + key);
  }, py::arg("key"), py::arg("value"), "set a native tuning entry (tests, A/B scripts)");
  m.def("set_fin_version", &set_fin_version,
        "BN finalize kernel variant: 0 = LDS tree, 2 = per-channel one-round, 1 = auto (default)");
  m.def("bn_acc_rep", []() { return BN_ACC_REP; }, "fp64 accumulator replicas per BatchNorm");
  m.def("prn_bar_words", &prn_bar_words, "32-bit words of the persistent step's barrier region (128-B aligned)");
  m.def("prn_acc_rep", &prn_acc_rep, "fp64 accumulator replicas per BatchNorm (persistent kernels)");
  m.def("pfin_cap", &pfin_cap, "max partials a consumer prologue combines for C channels");
  m.def("bn_bwd_tiles", &bn_bwd_tiles);
  m.def("bn_stats_tile_rows", &bn_stats_tile_rows);
  m.def("l2_workspace_floats", &l2_workspace_floats);
  m.def("softmax_xent_ws_floats", &softmax_xent_ws_floats);
  m.def("set_conv_parity", &set_conv_parity, py::arg("enabled"),
        "stride-2 dgrads as 4 output-parity classes (tune parity_dgrad)");
  m.def("set_conv_splitk", &set_conv_splitk, py::arg("max_slices"),
        "max split-K slices of under-filled implicit-GEMM grids (1 = off; tune splitk)");
  m.def("wgrad_reduce_chunks", &wgrad_reduce_chunks, py::arg("splits"), py::arg("K"),
        py::arg("taps"), py::arg("C"),
        "work chunks of one conv's slabs in wgrad_reduce_grouped (its desc's chunk0 stride)");
  m.def("wgrad_direct_bmp", [](std::vector<int> geom) { return wgrad_direct_bmp(geom_from(geom)); },
        "pixels per split of the direct 3x3 wgrad for this conv (0: the generic kernel runs)");
  m.def("wgrad_pick_splits", [](std::vector<int> geom) {
    int pps = 0;
    const int sp = wgrad_pick_splits(geom_from(geom), &pps);
    return py::make_tuple(sp, pps);
  });
  m.def("param_seg_bytes", []() { return (int)sizeof(ParamSeg); });
  m.def("wg_desc_bytes", []() { return (int)sizeof(WgReduceDesc); });
  m.def("opt_work_bytes", []() { return (int)sizeof(OptWork); });
  m.def("device_count", &hip_device_count);
  m.def("cu_count", &device_cus,
        "CUs this process dispatches to on the current device (the set bits of its CU mask, "
        "ROC_GLOBAL_CU_MASK; the device's CUs without one): persistent-grid sizing");
  m.def("cu_where", [](uint64_t out, int blocks, long long ticks, uint64_t stream) {
    cu_where(reinterpret_cast<unsigned*>(out), blocks, ticks, reinterpret_cast<hipStream_t>(stream));
  }, "diagnostics: per workgroup (HW_ID, XCC_ID) into out[2 * blocks] (CU-mask checks)");
  m.def("cu_mask", &device_cu_mask,
        "the process's CU mask on the current device as 32-bit words (bit i = CU i)");
  m.def(
      "crc32c",
      [](py::buffer b, uint32_t crc) {
        py::buffer_info info = b.request();
        // the byte count below assumes a dense C-contiguous buffer
        py::ssize_t expect = info.itemsize;
        for (int d = info.ndim - 1; d >= 0; --d) {
          if (info.shape[d] > 1 && info.strides[d] != expect)
            throw std::invalid_argument("crc32c: buffer must be C-contiguous");
          expect *= info.shape[d];
        }
        const size_t n = (size_t)info.size * (size_t)info.itemsize;
        py::gil_scoped_release nogil;
        return dtr::crc32c_extend(crc, reinterpret_cast<const uint8_t*>(info.ptr), n);
      },
      py::arg("data"), py::arg("crc") = 0);
  m.def("device_synchronize", []() {
    py::gil_scoped_release nogil;
    return (int)hipDeviceSynchronize();
  });
}
