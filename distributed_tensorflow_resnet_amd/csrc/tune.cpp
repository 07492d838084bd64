// Tuning registry (see tune.h).  Every default below was chosen by measurement on
// MI355X; the doc string names the measurement (profiles/, README "Tuning").
#include "tune.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

namespace dtr {

namespace {

// one entry per TuneId, in the enum order of tune.h
const TuneEntry kTable[T_COUNT] = {
    {"conv_pipe", 1,
     "2-deep pipelined (FAST) implicit-GEMM / wgrad loops where they pay: K loops >= 4 tiles, "
     "fwd >= 128 output channels, dgrad >= 16k rows (1.02-1.24x on the ImageNet shapes)"},
    {"splitk", 2,
     "max split-K slices of FAST grids with <= splitk_tiles tiles (the 7x7 stage: 196 tiles "
     "for 256 CUs)"},
    {"splitk_tiles", 256,
     "largest grid (tiles) that is split; splitting the 392-tile 14x14 grids measured slower "
     "(ImageNet step 12.93 -> 13.24 ms)"},
    {"dgrad_splitk", 1, "the 7x7 dgrads take the FAST loop once split-K doubles their grid"},
    {"nbuf1_kt", 1,
     "single-buffered LDS for K loops of <= this many 64-wide tiles: the 64-channel 1x1 convs "
     "fit 4 workgroups per CU instead of 2"},
    {"bm128_min", 4096,
     "rows from which >= 128-column convs use 128x128 tiles (7x7 fwd 118 -> 87 us)"},
    {"parity_dgrad", 1,
     "stride-2 dgrads as 4 output-parity classes of dense implicit GEMMs (3-3.5x faster than "
     "masked taps)"},
    {"direct_conv", 1, "direct halo 3x3 conv kernel for the CIFAR shapes (16@32, 32@16, 64@8)"},
    {"direct_splitn", -1,
     "column-split mask of the direct conv (bit 0: 32 ch, 1: 64 ch in 2, 2: 64 ch in 4); -1 "
     "auto by grid size"},
    {"direct_ldsw", 4,
     "direct conv weights staged through LDS, mask (1: 16 ch, 2: 32, 4: 64); C64 only: bs16 "
     "step 0.978 -> 0.955 ms"},
    {"direct_wgrad", 1, "direct halo wgrad for the CIFAR 3x3 shapes"},
    {"wgd_wt", 1,
     "direct wgrad split partials stored write-through (bs128 step 1.315 -> 1.302 ms)"},
    {"wgrad_target_wg", 768,
     "split-K wgrad: target workgroups (3 per CU hide the per-tile load latency)"},
    {"wgrad_slab_mb", 16,
     "split-K wgrad: cap of one layer's fp32 partial slabs, MB (RN50 bs128, back to back: "
     "32 10.68 / 10.70 ms, 16 10.62 / 10.60, 12 10.79, 8 11.38)"},
    {"fin_v", 1,
     "BN finalize variant: 1 auto (per-channel one-round kernel for many partials), 0 LDS "
     "tree, 2 one-round"},
    {"bwd_apply_fin", 1,
     "BN backward apply finalizes in-kernel: 0 only C <= 64, 1 when the redundant reads stay "
     "<= 1/4 of the streamed bytes, 2 always"},
    {"wt_store", -1,
     "conv epilogue write-through stores: -1 auto (direct convs writing >= 2 MB: bs128 step "
     "1.304 -> 1.282 ms; implicit-GEMM / ring convs always: RN50 bs128 10.32 -> 10.27 ms), "
     "0 off, 1 on"},
    {"plan_event_scope", 2,
     "plan fork/join events: 0 runtime default (system-scope release), 1 device-scope "
     "release, 2 no marker fence (CIFAR RN50 bs128 1.305 -> 1.280 ms, bs16 0.951 -> 0.932; "
     "1 = 0)"},
    {"wgrad_xcd", 1,
     "XCD-aware block order of the split-K weight gradients (RN50 bs128 wgrads 4.31 -> 4.11 "
     "ms/step in-process, step 12.18 -> 12.09 ms)"},
    {"ring_wgrad", 1,
     "LDS-DMA ring weight gradient (conv_wgrad_ring.hip) for the 128x128 tiles (RN50 bs128 "
     "wgrad kernels 4.68 -> 4.59 ms/step: no-PRE -5 %, PRE ties)"},
    {"ring", 1,
     "LDS-DMA ring implicit GEMM (conv_ring.hip) for the 128-row non-PRE convs (RN50 bs128 "
     "conv dgrads 4.51 -> 4.05 ms/step, forwards 3.94 -> 3.85)"},
    {"ring_kt", 5,
     "ring forwards from this many 64-deep K tiles (the 4-tile 14x14 256->1024 "
     "forward: 56 -> 61 us on the ring)"},
    {"ring_kt_dgrad", 4,
     "ring dgrads from this many 64-deep K tiles (the 4-tile 14x14 1024->256 dgrad: 75.8 -> "
     "68.8 us on the ring)"},
    {"prn_shards", -1,
     "arrival-counter shards (one 128-B line each, workgroup b on b % shards) of the persistent "
     "CIFAR step's grid barriers: -1 auto (64 when >= 128 slices of <= half an image arrive, "
     "else 8), or 1, 8, 16, 32, 64 (profiles/bn_barrier.md)"},
};

std::atomic<long> g_val[T_COUNT];
std::once_flag g_once;

std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && (s[a] == ' ' || s[a] == '\t')) ++a;
  while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t')) --b;
  return s.substr(a, b - a);
}

void load() {
  for (int i = 0; i < T_COUNT; ++i) g_val[i].store(kTable[i].dflt);
  const char* env = std::getenv("DTR_TUNE");
  if (!env) return;
  std::string s(env);
  size_t p = 0;
  while (p < s.size()) {
    size_t q = s.find(',', p);
    if (q == std::string::npos) q = s.size();
    const std::string item = s.substr(p, q - p);
    const size_t eq = item.find('=');
    if (eq != std::string::npos) {
      // keys and values trimmed like utils/tune.py; a value that is not a whole
      // integer is rejected loudly instead of being truncated by strtol
      const std::string k = trim(item.substr(0, eq));
      const std::string v = trim(item.substr(eq + 1));
      for (int i = 0; i < T_COUNT; ++i) {
        if (k != kTable[i].key) continue;
        char* end = nullptr;
        const long val = std::strtol(v.c_str(), &end, 10);
        if (v.empty() || end == nullptr || *end != '\0') {
          std::fprintf(stderr, "DTR_TUNE: %s=%s is not an integer; keeping the default %ld\n",
                       k.c_str(), v.c_str(), kTable[i].dflt);
          break;
        }
        g_val[i].store(val);
      }
      // keys of the Python engine (utils/tune.py) are validated there
    }
    p = q + 1;
  }
}

}  // namespace

long tune(TuneId id) {
  std::call_once(g_once, load);
  return g_val[id].load(std::memory_order_relaxed);
}

void tune_set(TuneId id, long v) {
  std::call_once(g_once, load);
  g_val[id].store(v);
}

const TuneEntry* tune_table() { return kTable; }

}  // namespace dtr
