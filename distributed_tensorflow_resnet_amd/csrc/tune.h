// Tuning registry of the native layer: every tile / schedule parameter that was
// chosen by measurement lives in ONE table (tune.cpp) with its default and the
// measurement behind it, instead of one environment variable per experiment.
//
// Overrides come from a single environment variable, read once:
//     DTR_TUNE="splitk=1,conv_pipe=0"
// (the same string also carries the Python engine's keys, utils/tune.py; an
// unknown key is an error there).  Tests flip entries with tune_set().  README.md
// "Tuning" documents every key with its default (tests/test_tune_cpu.py checks).
#pragma once

namespace dtr {

enum TuneId : int {
  T_CONV_PIPE = 0,     // pipelined FAST loops (conv / wgrad)
  T_SPLITK,            // max split-K slices of under-filled FAST grids
  T_SPLITK_TILES,      // largest grid (tiles) that is split
  T_DGRAD_SPLITK,      // 7x7 dgrads: FAST loop once split-K doubles their grid
  T_NBUF1_KT,          // single-buffered LDS for K loops of <= this many tiles
  T_BM128_MIN,         // rows from which 128x128 tiles are used (>= 128 columns)
  T_PARITY_DGRAD,      // stride-2 dgrads as 4 output-parity classes
  T_DIRECT_CONV,       // direct halo 3x3 kernel for the CIFAR shapes
  T_DIRECT_SPLITN,     // its column-split mask (-1 auto)
  T_DIRECT_LDSW,       // its weight staging through LDS, mask of C16/C32/C64
  T_DIRECT_WGRAD,      // direct halo wgrad for the CIFAR shapes
  T_WGD_WT,            // its split partials stored write-through
  T_WGRAD_TARGET_WG,   // split-K wgrad: target workgroups
  T_WGRAD_SLAB_MB,     // split-K wgrad: cap of one layer's fp32 partial slabs (MB)
  T_FIN_V,             // BN finalize kernel variant (-1 auto)
  T_BWD_APPLY_FIN,     // BN backward apply finalizes in-kernel when the grid allows
  T_WT_STORE,          // conv epilogue write-through stores (-1 auto, 0 off, 1 on)
  T_PLAN_EVENT_SCOPE,  // release scope of the plan's fork/join events
  T_WGRAD_XCD,         // XCD-aware block order of the split-K weight gradients
  T_RING_WGRAD,        // LDS-DMA ring weight gradient (conv_wgrad_ring.hip), 128x128 tiles
  T_RING,              // LDS-DMA ring implicit GEMM (conv_ring.hip) for eligible convs
  T_RING_KT,           // ... forward convs with K loops of at least this many 64-deep tiles
  T_RING_KT_DGRAD,     // ... dgrads with K loops of at least this many tiles
  T_PRN_SHARDS,        // arrival-counter shards of the persistent CIFAR step's grid barriers
  T_COUNT
};

struct TuneEntry {
  const char* key;
  long dflt;
  const char* doc;
};

long tune(TuneId id);               // current value (DTR_TUNE override or default)
void tune_set(TuneId id, long v);   // tests / A-B scripts
const TuneEntry* tune_table();      // T_COUNT entries, indexed by TuneId

}  // namespace dtr
