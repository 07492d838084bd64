// Host-visible launcher interface of the gfx950 kernel library.  Every launcher
// takes raw device pointers plus an explicit hipStream_t, performs no
// allocation and no synchronisation, and is therefore safe inside hipGraph
// stream capture (the whole training step is captured; see train/engine.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "tune.h"

namespace dtr {

typedef __bf16 bf16;

// fp64 accumulator replicas per BatchNorm of the per-layer kernels (replica =
// blockIdx % REP: two XCDs each).  Same-box A/B, ImageNet RN50 bs128 / per-layer CIFAR
// bs128 step ms (profiles/bn_acc_replicas.md): 2: 10.48 / 1.429, 4: 10.47 / 1.298,
// 8: 10.54 / 1.267, 16: 10.72 / 1.266 -- 4 for the ImageNet headline (the per-layer
// CIFAR path only runs above 240 images per rank; the persistent step uses its own count)
constexpr int BN_ACC_REP = 4;

enum { MODE_FWD = 0, MODE_DGRAD = 1 };

struct ConvGeom {
  int N, H, W, C;     // input activation (NHWC)
  int Ho, Wo, K;      // output spatial dims, output channels
  int kh, kw, stride, pad;
};

// Fused BatchNorm finalize in the producing kernel (last-arriver; see bn_fused.h).
struct BnFwdFin {            // forward statistics -> mean/rstd/scale/shift + moving averages
  unsigned* counters;        // [col tiles] level-2 (or only) + [col tiles][groups] level-1;
                             // nullptr = disabled
  const float* gamma;
  const float* beta;
  float* mmean;
  float* mvar;
  float* mean;
  float* rstd;
  float* scale;
  float* shift;
  float momentum, eps;
  int update_moving;
  float* gpart;              // two-level: [groups][2][NC] group partials (mean, M2)
  int group;                 // tiles per level-1 group; 0 = single level
  int groups_only;           // 1: stop after level 1 (a consumer's BnPreFin combines gpart)
};
// Consumer-side BN finalize: the FIRST kernel that applies a BN (the next conv's
// fused BN+ReLU prologue) combines the producer's (mean, M2) partials itself --
// every workgroup redundantly into its LDS scale/shift table, block (0,0) also
// writing mean/rstd/scale/shift and the moving averages for later consumers --
// so no separate finalize launch sits between producer and consumer.
struct BnPreFin {
  const float* part;         // [cnt][2][C] (mean, M2); cnt == 0 -> disabled
  int cnt;                   // acc mode: 1
  const double* acc;         // optional [BN_ACC_REP][2][C] (sum y, sum y^2): replaces part
  int rows_per;              // rows per partial (the last one holds the remainder)
  int M;                     // rows in total
  const float* gamma;
  const float* beta;
  float* mean;
  float* rstd;
  float* scale;
  float* shift;
  float* mmean;
  float* mvar;
  float momentum, eps;
  int update_moving;
};
struct BnBwdFin {            // backward sums -> dgamma/dbeta/apply coefficients
  unsigned* counters;        // nullptr = disabled
  const float* gamma;
  const float* rstd;
  float* dgamma;
  float* dbeta;
  float* coef;               // [3][C]
  float* gpart;              // two-level: [groups][2][NC] group sums
  int group;                 // tiles per level-1 group; 0 = single level
  int groups_only;           // 1: stop after level 1 (a consumer's BnBwdPre combines gpart)
};
// Consumer-side BatchNorm+ReLU backward (direct dgrad only): the dgrad's A operand
// is the BN-backward output dh = a*g - b - c*xhat (+ add), g = da*[x*scale+shift > 0],
// computed while staging the halo from da (GemmArgs::a), x and add; the (sum g,
// sum g*xhat) partials of the producer are combined in the prologue (coefficients a,
// b, c); the interior of the halo (this tile's dh rows) is written to a_out for the
// other consumers (wgrad, residual path); block (0,0) writes dgamma/dbeta/coef.
struct BnBwdPre {
  const bf16* x;             // BN input [M][C]; nullptr = disabled
  const bf16* add;           // optional gradient added to dh (residual branch)
  const float* mean;
  const float* rstd;
  const float* scale;
  const float* shift;
  const float* gamma;
  const float* part;         // [cnt][2][C] (sum g, sum g*xhat)
  int cnt;                   // acc mode: 1
  const double* acc;         // optional [BN_ACC_REP][2][C] (sum g, sum g*xhat): replaces part
  bf16* a_out;               // dh [M][C]
  float* dgamma;
  float* dbeta;
  float* coef;               // [3][C]
};

struct GemmArgs {
  const bf16* a;            // x (fwd) or dy (dgrad), NHWC
  const bf16* b;            // weights: [K][kh][kw][C] (fwd) or [kh][kw][C][K] (dgrad)
  bf16* out;                // [M][Ncol] bf16 (unless out_f32)
  float* out_f32;           // optional fp32 output
  const bf16* residual;     // optional [M][Ncol] residual added in the epilogue
  const float* pre_scale;   // optional per-A-channel BN scale (fused BN+ReLU on load)
  const float* pre_shift;
  const float* bias;        // optional, applied to columns < nbias
  int nbias;
  float* stat_part;         // optional [tiles][2][Ncol] Welford partials (mean, M2)
  // optional fused BN+ReLU backward reduction (dgrad): x = BN input [M][Ncol]
  const bf16* bnb_x;
  const float* bnb_mean;
  const float* bnb_rstd;
  const float* bnb_scale;
  const float* bnb_shift;
  float* bnb_part;          // [tiles][2][Ncol]: sum g, sum g*xhat
  BnFwdFin fin;             // with stat_part: finalize in-kernel
  BnBwdFin bfin;            // with bnb_part: finalize in-kernel
  // Accumulator mode of STATS / BNB: instead of (or beside) the per-tile partials,
  // every workgroup adds its tile's sums into [BN_ACC_REP][2][Ncol] fp64 replicas
  // (replica = blockIdx.x % BN_ACC_REP) with memory-side atomics, so
  // a consumer reads 2 x BN_ACC_REP values per channel instead of combining every
  // tile partial.  The buffers are zeroed once per step.
  double* stat_acc;         // STATS: sum y, sum y^2
  double* bnb_acc;          // BNB: sum g, sum g*xhat
  BnPreFin pfin;            // with pre_scale: finalize the PRE BatchNorm in the prologue
  BnBwdPre abwd;            // direct dgrad: BN backward on the A operand (see above)
  int accumulate;           // out += result
  ConvGeom g;
  int M, Ncol, Kdim;
  long long* probe = nullptr;   // direct conv: per-workgroup phase timestamps (diagnostics)
  int wt = 0;                   // epilogue output stores write-through (sc1): tune wt_store
  // split-K (conv_gemm FAST loop; set by the launcher): gridDim.z = ksplit slices of the
  // K tiles; each slice publishes its fp32 tile to sk_part, the last arriver of the tile
  // (sk_cnt) sums the slices in slice order and runs the epilogue
  int ksplit = 1;
  float* sk_part = nullptr;
  unsigned* sk_cnt = nullptr;
  // stride-2 dgrad by output parity class (conv_gemm; set by the launcher): gridDim.z = 4
  // classes (h+pad, w+pad) mod 2, each a dense GEMM over its own rows and only the filter
  // taps that reach them.  par != 0 enables it; the kernel fills in its class's row
  // geometry (first row / column, rows / columns per image) for the epilogue.
  int par = 0;
  int par_h0 = 0, par_w0 = 0, par_hc = 0, par_wc = 0;
};

// Streaming 1x1 dgrad with a narrow reduction (K = 64..256) fused with the BN+ReLU
// backward of its wide output (bn_dgrad1x1.hip): mode 0 sums (sum g, sum g*xhat) into
// bacc, mode 1 writes dx = a*g - b - c*xhat (+ add) with coef = (a, b, c).
struct BndArgs {
  const bf16* dz;           // [M][K] the 1x1 conv's output gradient
  const bf16* w;            // [C][K] dgrad weights (HWIO of the 1x1 conv)
  const bf16* x;            // [M][C] BN input
  const bf16* add;          // optional [M][C] added to dx (mode 1)
  bf16* out;                // [M][C] dx (mode 1)
  const float* mean;
  const float* rstd;
  const float* scale;
  const float* shift;
  const float* coef;        // [3][C] (mode 1)
  double* bacc;             // [BN_ACC_REP][2][C] (mode 0)
  int M, C, K;
};
bool bnd1x1_covers(int M, int C, int K);
void bnd1x1(const BndArgs& a, int mode, hipStream_t s);

// Streaming 1x1 forward conv with a narrow reduction (K = 64..256) and a wide output
// (bn_fwd1x1.hip): y = bf16(relu(bn(x)) W^T + res), BN statistics of y into stat_acc.
struct BnfArgs {
  const bf16* x;            // [M][K] input (pre-BN when PRE)
  const bf16* w;            // [C][K] OHWI weights of the 1x1 conv
  const bf16* res;          // optional [M][C] residual
  bf16* out;                // [M][C]
  const float* pre_scale;   // optional BN+ReLU of x (finalized) ...
  const float* pre_shift;
  BnPreFin pfin;            // ... or finalized here from fp64 accumulators (pfin.acc)
  double* stat_acc;         // optional [BN_ACC_REP][2][C] (sum y, sum y^2)
  int M, C, K;
};
bool bnf1x1_covers(int M, int C, int K);
void bnf1x1(const BnfArgs& a, hipStream_t s);

void conv_gemm(const GemmArgs& a, int mode, hipStream_t s);
// Split-K slab bytes (and tile counters) conv_gemm would use for this conv, 0 = none;
// launches nothing.  Plans size their per-stream workspace with it at record time.
size_t conv_gemm_splitk_need(const GemmArgs& a, int mode, size_t* tiles);
void set_conv_splitk(int max_slices);   // split-K of under-filled FAST grids (1 = off)
void set_conv_parity(int enabled);      // stride-2 dgrads by output parity class
// Direct halo-tiled 3x3/s1 kernel for small C (conv_direct.hip); false = not covered.
bool conv_direct(const GemmArgs& a, int mode, hipStream_t s);
bool conv_direct_covers(const GemmArgs& a, int mode);
void set_direct_probe(long long* p);   // per-workgroup phase stamps of the direct conv (diag)
void plan_delay(long long ticks, hipStream_t s);   // spin one wave for ticks x 10 ns (diag.hip)
// per workgroup (HW_ID, XCC_ID) into out[2 * blocks], each spinning ticks x 10 ns (diag.hip)
void cu_where(unsigned* out, int blocks, long long ticks, hipStream_t s);
void set_conv_direct(int enabled);
void set_conv_pipeline(int enabled);   // 2-deep pipelined implicit-GEMM / wgrad loops (tune conv_pipe)
void set_fin_version(int v);   // BN finalize kernel variant (tune fin_v)
int conv_gemm_bm(int M, int Ncol);
// LDS-DMA ring loop (conv_ring.hip) for the 128x128 non-PRE tiles: covers / launch on the
// caller's grid (split-K / parity set up by the caller, conv_gemm.hip)
bool conv_ring_covers(const GemmArgs& a, int mode);
void conv_ring(const GemmArgs& a, int mode, int flags, dim3 grid, hipStream_t s);
bool conv_gemm_uses_ring(const GemmArgs& a, int mode);
int conv_gemm_bn(int M, int Ncol);   // column tile of the kernel conv_gemm() picks

// ---- Persistent small-batch CIFAR step (cifar_persist.hip) ----
// The whole CIFAR ResNet v2 (6n+2, building blocks, 16/32/64 channels on 32/16/8 maps;
// resnet_model_official.py:217-278) forward in ONE launch and its backward in ONE
// launch.  Each image is split into P row slices, one 512-thread workgroup per slice,
// that keep their activations on-chip across layers; the two halo rows a 3x3 conv needs
// from the neighbouring slices come from tensors the neighbours publish anyway (the
// saved activations, the backward's gradients); grid barriers only where BatchNorm
// needs batch statistics (exact fp64 atomic sums).  In the backward launch the
// remaining CUs compute the weight gradients (per image group, fp32 slabs for the
// grouped reduce) as soon as the slices have published each layer's output gradient.
struct PrnBn {               // one BatchNorm (all device pointers)
  const float* gamma;
  const float* beta;
  float* mmean;              // moving statistics (updated by workgroup 0)
  float* mvar;
  float* mean;               // batch statistics (written by workgroup 0)
  float* rstd;
  float* scale;
  float* shift;
  float* dgamma;             // gradients in the flat fp32 gradient buffer (workgroup 0)
  float* dbeta;
  double* acc;               // [BN_ACC_REP][2][C] forward sums (sum y, sum y^2), zeroed per step
  double* bacc;              // [BN_ACC_REP][2][C] backward sums (sum g, sum g xhat)
};
struct PrnBlock {            // one building block (resnet_model_official.py:94-130)
  bf16* x;                   // block input [N][R_in][R_in][C_in], NHWC (saved, published)
  bf16* h1;                  // conv1 output [N][R][R][C] (saved, published)
  bf16* out;                 // block output (the next block's x)
  const bf16* w1f;           // forward weights, OHWI [co][kh][kw][ci]
  const bf16* w2f;
  const bf16* wpf;           // projection shortcut (nullptr: identity)
  const bf16* w1b;           // dgrad weights, HWIO [kh][kw][ci][co]
  const bf16* w2b;
  const bf16* wpb;
  bf16* dout;                // backward: gradient of `out` (published)
  bf16* dh1;                 // backward: gradient of h1 after BN2's backward (published)
  bf16* da2;                 // backward: conv2's dgrad output, before BN2's backward (published)
  bf16* da1;                 // backward: conv1's (+ projection's) dgrad output (published)
  int stage;                 // output stage 0..2 (32x32x16, 16x16x32, 8x8x64)
  int stride;                // 1 or 2 (the first block of stages 1 and 2)
  int bn1, bn2;              // PrnBn indices of the block's two BatchNorms
};
struct PrnItem {             // backward weight-gradient work item: one conv x one image group
  const bf16* dy;            // [N][Ro][Ro][CO] output gradient (published by the slices)
  const bf16* x;             // [N][Ri][Ri][CI] conv input before its BatchNorm (stem: the image)
  const float* scale;        // BN+ReLU of x (nullptr: none -- the stem)
  const float* shift;
  float* part;               // [CO][taps*CI] fp32 slab of this image group
  int kind;                  // conv shape class (prn_item_kind)
  int img0, nimg;
  int ready;                 // backward barrier arrivals (x slices) after which dy is complete
  int bucket;                // overlap mode: all-reduce bucket whose counter counts this item
                             // (its slab stored write-through), -1 none
  int pad_;
};
struct PrnArgs {
  const PrnBlock* blocks;
  int nblocks;
  const PrnBn* bns;          // [2 * nblocks + 1]: block i's BNs at 2i, 2i + 1; the final BN last
  const bf16* x_in;          // [N][32][32][8] input images (channels 3..7 zero)
  const bf16* stem_w;        // OHWI [16][3][3][8]
  double* pool_acc;          // [N][64] fp64 average-pool sums (zeroed every step)
  unsigned* bar;             // [prn_bar_words()], 128-B aligned: sharded arrival counters
                             // (forward, backward), the backward readiness count and the
                             // weight-gradient item queue, each on its own lines -- zeroed
                             // every step (cifar_persist.hip PRN_FWD .. PRN_QUEUE)
  int* err;                  // set when a barrier wait times out
  const bf16* dense_w;       // [64][kpad] bf16 HWIO
  const float* dense_b;
  const int* labels;
  bf16* pooled;              // [N][64]
  bf16* dlogits;             // [N][kpad]
  float* ws;                 // softmax_xent workspace: [N][kpad] gradient rows, then [N][2]
  float* dpool;              // [N][64] fp32: average-pool gradient per channel (dact)
  // the head's batch folds (prn_head):
  float* loss_sum;           // sum of the per-image losses
  float* correct;            // number of correct top-1 predictions
  float* dbias;              // [classes] dense bias gradient
  float* dense_grad;         // [64][classes] fp32 dense weight gradient (HWIO)
  bf16* dx0;                 // backward: gradient of the stem output [N][32][32][16]
  const PrnItem* items;      // backward weight-gradient items, in readiness order
  int nitems;
  int N, P, classes, kpad;   // P: row slices (workgroups) per image
  float grad_scale;          // 1 / global batch
  float momentum, eps;
  int update_moving;
  long long* probe = nullptr;   // diagnostics: workgroup 0's (tag, wall clock) phase stamps
  int shards = 8;            // arrival-counter shards (tune prn_shards: 1 or 8)
  // overlap mode (world > 1): each weight-gradient item's slab is stored write-through
  // and counted on its bucket's line of `bar` (PRN_BUCKET), and slice workgroup 0 counts
  // the bucket's BatchNorm gradients there once its last BN backward is stored, so the
  // comm stream's slab reduce + all-reduce of a bucket start while the backward runs
  int overlap = 0;
  int bucket_of_stage[3] = {-1, -1, -1};   // stage 0..2 -> bucket (overlap mode)
  int fault_bar = -1;        // tests only (DTR_PRN_FAULT_BAR): forward workgroup 0 abandons the
                             // launch at this barrier, as a lost workgroup would; -1 off
};
enum { PRN_THREADS = 512 };
void prn_set_probe(long long* p);   // diagnostics (scripts/prn_probe.py); nullptr = off
bool prn_supported(int N, int P, int nblocks, int classes, int kpad);
// Every host-side limit of the three persistent launches at once (forward at P_fwd slices,
// backward at P, the head folds), including co-residency from the occupancy API: "" when
// the step is supported, else the reason.  The engine calls it once when it builds the plan.
std::string prn_check(int N, int P, int P_fwd, int nblocks, int classes, int kpad);
// CUs this process dispatches to on the current device (its CU mask's set bits) and the mask
int device_cus();
std::vector<uint32_t> device_cu_mask();
size_t prn_lds_bytes();
int prn_bar_words();   // barrier / readiness / queue words of PrnArgs::bar (zeroed every step)
int prn_acc_rep();   // fp64 accumulator replicas per BatchNorm of the persistent kernels
void prn_forward(const PrnArgs& a, hipStream_t s);
void prn_backward(const PrnArgs& a, int wgrad_wgs, hipStream_t s);
// the head's batch folds (loss, precision, dense bias + weight gradients), one workgroup
void prn_head(const PrnArgs& a, hipStream_t s);
// comm-stream wait (overlap mode): one wave polls bar[PRN_BUCKET + 32 b] until it reaches
// `target` (bounded: 2 s, then *err), so the launches behind it on that stream start once
// bucket b's gradients are complete
void prn_bucket_wait(unsigned* bar, int bucket, unsigned target, int* err, hipStream_t s);
// item kind of a conv (stage of its output, kernel size, stride; stem = 8 input channels)
int prn_item_kind(int cin, int cout, int ksize, int stride);

struct WgradArgs {
  const bf16* dy;           // [N,Ho,Wo,K]
  const bf16* x;            // [N,H,W,C] (pre-BN tensor if pre_scale given)
  const float* pre_scale;   // optional fused BN+ReLU on x
  const float* pre_shift;
  float* part;              // [splits][K][kh*kw*C] fp32 partials
  ConvGeom g;
  int splits;
  int px_per_split;         // multiple of 64
  int wt = 0;               // partials stored write-through (direct kernel; set by the launcher)
  int xcd = 0;               // 1: XCD-aware block order (the column tiles of one split share an L2)
};
// LDS-DMA ring weight gradient (conv_wgrad_ring.hip): 128 x 128 tiles, same splits / slabs
bool conv_wgrad_ring_covers(const WgradArgs& a);
void conv_wgrad_ring(const WgradArgs& a, hipStream_t s);

void conv_wgrad(const WgradArgs& a, hipStream_t s);
// Direct halo-tiled wgrad for 3x3/s1 small C (conv_wgrad_direct.hip).
bool conv_wgrad_direct(const WgradArgs& a, hipStream_t s);
int wgrad_direct_bmp(const ConvGeom& g);   // pixels per split, 0 = not covered
void set_wgrad_direct(int enabled);
// grad[tap][ci][co] (+)= scale * sum_s part[s][co][tap*C+ci] for co < K_valid, ci < C_valid
// (output is the unpadded TF HWIO tensor [taps][C_valid][K_valid])
void wgrad_reduce(const float* part, float* grad_hwio, int splits, int K, int K_valid, int taps,
                  int C, int C_valid, float scale, int accumulate, hipStream_t s);
int wgrad_pick_splits(const ConvGeom& g, int* px_per_split);

struct WgReduceDesc {      // one convolution's split-K slabs -> its HWIO gradient
  const float* part;       // [splits][K][taps*C]
  float* grad;             // [taps][Cv][Kv]
  int splits, K, Kv, taps, C, Cv;
  long long chunk0;        // first 64-column work chunk of this conv in the group
};
void wgrad_reduce_grouped(const WgReduceDesc* descs_dev, int nd, long long total_chunks,
                          float scale, hipStream_t s);
// work chunks of one conv in a grouped reduce (its desc's chunk0 advances by this)
long long wgrad_reduce_chunks(int splits, int K, int taps, int C);

// ---- BatchNorm (training mode, TF fused semantics) ----
void bn_finalize(const float* stat_part, int tiles, int tile_rows, int M, int C,
                 const float* gamma, const float* beta, float* moving_mean,
                 float* moving_var, float momentum, float eps, int update_moving,
                 float* mean, float* rstd, float* scale, float* shift, hipStream_t s);
// Accumulator-mode finalizers (acc = [BN_ACC_REP][2][C] fp64 sums, see GemmArgs).
void bn_finalize_acc(const double* acc, int M, int C, const float* gamma, const float* beta,
                     float* moving_mean, float* moving_var, float momentum, float eps,
                     int update_moving, float* mean, float* rstd, float* scale, float* shift,
                     hipStream_t s);
void bn_bwd_finalize_acc(const double* acc, int M, int C, const float* gamma, const float* rstd,
                         float* dgamma, float* dbeta, float* coef, hipStream_t s);
void bn_scale_shift_eval(const float* gamma, const float* beta, const float* moving_mean,
                         const float* moving_var, float eps, int C, float* scale,
                         float* shift, hipStream_t s);
// per-channel reductions for BN+ReLU backward: sum(g), sum(g*xhat) with g = dy*[y>0]
void bn_relu_bwd_reduce(const bf16* dy, const bf16* x, const float* mean, const float* rstd,
                        const float* scale, const float* shift, int M, int C, float* part,
                        int* tiles_out, hipStream_t s);
int bn_bwd_tiles(int M, int C);
// finalize: dgamma, dbeta (added to grads), coefficients for apply
void bn_bwd_finalize(const float* part, int tiles, int M, int C, const float* gamma,
                     const float* rstd, float* dgamma, float* dbeta, float* coef,
                     hipStream_t s);
// dx = coef_a*g - coef_b - coef_c*xhat (+ residual-grad add)
void bn_relu_bwd_apply(const bf16* dy, const bf16* x, const float* mean, const float* rstd,
                       const float* scale, const float* shift, const float* coef,
                       const bf16* add, bf16* dx, int M, int C, hipStream_t s);
// acc-mode BN finalize + materializing BN+ReLU pass in one launch (bn.hip)
void bn_relu_apply_acc(const bf16* x, bf16* y, int M, int C, const double* acc,
                       const float* gamma, const float* beta, float* moving_mean,
                       float* moving_var, float momentum, float eps, int update_moving,
                       float* mean, float* rstd, float* scale, float* shift, hipStream_t s);
void bn_relu_apply(const bf16* x, const float* scale, const float* shift, bf16* y, int M,
                   int C, hipStream_t s);
// The same apply with the finalize fused in (accumulator mode, small C): every block
// derives the coefficients from the fp64 sums; block 0 writes dgamma/dbeta/coef.
constexpr int BWD_ACC_FIN_MAXC = 64;
struct BwdAccFin {
  const double* acc;        // [BN_ACC_REP][2][C] (sum g, sum g*xhat); nullptr = off
  const float* gamma;
  float* dgamma;
  float* dbeta;
  float* coef;              // [3][C] out
  int M;
};
bool bn_bwd_apply_acc_fits(int M, int C);
void bn_relu_bwd_apply_acc(const bf16* dy, const bf16* x, const float* mean, const float* rstd,
                           const float* scale, const float* shift, const BwdAccFin& fin,
                           const bf16* add, bf16* dx, int M, int C, hipStream_t s);

void bn_stats(const bf16* x, int M, int C, float* part, hipStream_t s);
int bn_stats_tile_rows();

// ---- head: BN-ReLU + global average pool, softmax cross-entropy ----
void bnrelu_avgpool(const bf16* x, const float* scale, const float* shift, bf16* pooled,
                    int N, int HW, int C, hipStream_t s);

// Whole training head in one launch (small heads: C <= 64 channels, HW <= 64, <= 64
// padded classes -- the CIFAR networks): final BN finalize from its fp64
// accumulators, BN+ReLU + global average pool, dense + bias, softmax cross-entropy
// rows (per-row loss / correct / gradient into the softmax_xent workspace),
// dense data gradient, average-pool backward (writes dact) and the final BN's
// backward sums into its fp64 accumulators.  One workgroup per image.  The
// batch-level folds (loss, precision, dbias) are softmax_xent_reduce's, the dense
// weight gradient conv_wgrad's -- both off the critical path.
struct HeadArgs {
  const bf16* x;            // [N][HW][C] final BN input
  const double* acc;        // final BN forward accumulators [BN_ACC_REP][2][C]
  const float* gamma;
  const float* beta;
  float* mmean;
  float* mvar;
  float* mean;              // outputs (block 0): mean, rstd, scale, shift
  float* rstd;
  float* scale;
  float* shift;
  float momentum, eps;
  int update_moving;
  const bf16* w;            // dense weights, bf16 HWIO [C][kpad] (padded columns zero)
  const float* bias;        // [classes]
  const int* labels;        // [N]
  int N, HW, C, classes, kpad;
  float grad_scale;         // 1 / global batch
  bf16* pooled;             // [N][C]
  bf16* dlogits;            // [N][kpad]
  float* ws;                // softmax_xent workspace: [N][kpad] fp32 gradient rows, [N][2]
  bf16* dact;               // [N][HW][C] gradient of the pooled activations
  double* bacc;             // final BN backward accumulators (sum g, sum g*xhat)
};
bool head_fused_supported(int N, int HW, int C, int classes, int kpad);
void head_fused(const HeadArgs& a, hipStream_t s);
void softmax_xent_reduce(const float* ws, int ld, int N, int classes, float* loss_sum,
                         float* correct, float* dbias, hipStream_t s);
void avgpool_bwd(const bf16* dpooled, bf16* dx, int N, int HW, int C, hipStream_t s);
void softmax_xent(const float* logits, int ld, const int* labels, int N, int classes,
                  float* loss_sum, float* correct, bf16* dlogits, float* dbias,
                  float grad_scale, float* probs, float* ws, hipStream_t s);
long softmax_xent_ws_floats(int N, int ld);

// ---- max pool (ImageNet stem) ----
void maxpool_fwd(const bf16* x, bf16* y, uint8_t* argmax, int N, int H, int W, int C, int Ho,
                 int Wo, int k, int stride, int pad, hipStream_t s);
void maxpool_bwd(const uint8_t* argmax, const bf16* dy, bf16* dx, int N, int H, int W, int C,
                 int Ho, int Wo, int k, int stride, int pad, hipStream_t s);

// ---- flat-parameter descriptors ----
struct ParamSeg {          // one trainable tensor inside the flat buffers
  long long offset;        // element offset into master/grad/mom (master layout = TF HWIO)
  long long numel;
  long long bf_ohwi;       // element offset of the bf16 [Kpad][kh][kw][Cpad] copy (-1: none)
  long long bf_hwio;       // element offset of the bf16 [kh][kw][C][Kpad] copy (-1: none)
  int kh, kw, C, K;        // geometry of the master tensor (kh=kw=1 for dense)
  int cpad;                // padded input channels of the OHWI copy
  int kpad;                // padded output channels of both copies
};

}  // namespace dtr
