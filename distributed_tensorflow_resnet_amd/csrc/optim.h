// Optimizer-side declarations (see optim.hip).
#pragma once
#include "kernels.h"

namespace dtr {

// Piecewise learning-rate schedule evaluated on the device from global_step.
struct LrSchedule {
  float init;            // rate used at step 0 (the hook's begin())
  long long warm_steps;  // linear warm-up length (0 = none)
  float warm_from, warm_to;
  int nb;                // number of boundaries (<= 7)
  long long bound[7];
  float val[8];
};

void sgd_update_pack(float* master, const float* grad, float* mom, long n, const LrSchedule& s,
                     const long long* gstep, float momentum, float wd, float grad_scale,
                     int use_momentum, const ParamSeg* segs, int nseg, bf16* bf, float* lr_out,
                     int update, hipStream_t st);
// OHWI bf16 weight copies by a tiled transpose of the fp32 master (after the update);
// gstep_inc (optional): global_step += 1 in the same launch.
void ohwi_pack(const float* master, const ParamSeg* segs, const long long* tile0, int nseg,
               long long total_tiles, bf16* bf, long long* gstep_inc, hipStream_t s);
// The fused optimizer of the persistent step (sgd_tiles): per parameter segment, the
// work map of one launch that (optionally) sums the split-K weight-gradient slabs,
// applies SGD-momentum + wd and writes both bf16 copies.
struct OptWork {
  const float* part;       // slabs [splits][K'][taps*cslab] (null: the gradient is in grad)
  long long tile0;         // first workgroup of the segment
  int splits, kslab;       // slab count and rows (output channels, padded) of a slab
  int cslab;               // padded input channels of a slab row (taps*cslab columns)
  int tiled;               // 1: tr (tap*C+ci) x tc (co) tiles; 0: 1024-element chunks
  int tr, tc;              // tile rows / columns (<= 64 each)
};
// blk_seg[b] = the segment of workgroup b; ticket: a zero-initialised int the last
// workgroup resets after its global_step += 1 (every workgroup has read the step); null:
// no global_step increment (a launch updating part of the parameters ahead of the last).
// gin (no slabs): the gradient read as bf16 from gin (the bf16 all-reduce's result; the
// fp32 grad is written from it).  pack: no update -- the gradient (slab sums or grad) is
// only written out, as bf16 to gout (or, gout null, as fp32 to grad): the all-reduce's
// input in one launch instead of a grouped reduce plus a cast.
void sgd_tiles(float* master, float* grad, float* mom, const LrSchedule& s, long long* gstep,
               float momentum, float wd, float grad_scale, int use_momentum,
               const ParamSeg* segs, const OptWork* work, const int* blk_seg, int nblocks,
               bf16* bf, float* lr_out, unsigned* ticket, const bf16* gin, bf16* gout, int pack,
               hipStream_t st);
void step_increment(long long* gstep, hipStream_t s);
int l2_workspace_floats();
void l2_half_sum(const float* v, long n, float* ws, float* out, hipStream_t s);
void fill_f32(float* p, long n, float a, hipStream_t s);
void cast_f32_bf16(const float* a, bf16* b, long n, hipStream_t s);
void cast_bf16_f32(const bf16* a, float* b, long n, hipStream_t s);

}  // namespace dtr
