"""Tuning entries of the training engine (plan schedule and fusion choices).

One environment variable carries every tuning override of the framework,
Python engine and native kernels alike:

    DTR_TUNE="fork_every=2,splitk=1"

The engine keys are below (read when an Engine is built); the native keys
(tile shapes, split-K, kernel variants) live in csrc/tune.h / tune.cpp, read
once per process (tests flip those with ``_C.tune_set``).  An unknown key is an
error.  README.md "Tuning" lists every key with its default; the CPU test
tests/test_tune_cpu.py checks that the list, the tables and the code agree.
"""
from __future__ import annotations

import os

# key: (default, meaning + the measurement behind the default)
ENGINE = {
    "fork_wgrad": (-1, "weight gradients on the side stream: 1 on, 0 all on the main stream, "
                       "-1 auto (on eagerly; off under hipGraph capture, which replays the "
                       "cross-stream event edges poorly)"),
    "fork_every": (-1, "residual blocks per side-stream fork, -1 auto: 4 CIFAR (bs16 0.948 vs "
                       "0.959 / 1.012 ms at 2 / 8), 2 ImageNet (12.81 vs 12.91 ms at 4)"),
    "tail_main": (-1.0, "fraction of the backward tail's queued weight gradients run on the "
                        "idle main stream after the stem, -1 auto: 1 CIFAR (bs128 1.326 -> 1.303 "
                        "ms at 0 -> 1), 0.5 ImageNet (RN50 10.56 -> 10.49 ms, RN101 32.78 -> "
                        "32.66 ms at 1 -> 0.5)"),
    "reduce_main_tail": (1, "the last split-K reduces run on the main stream behind one join"),
    "reduce_mb": (-1.0, "split-K reduce group size in MB, -1 auto (~6 groups, <= 4 MB: CIFAR "
                        "RN50 -2.3 % step vs one group)"),
    "stem_s2d": (1, "ImageNet 7x7/2 stem as a space-to-depth 4x4/1 conv (K 392 -> 256)"),
    "bn_acc": (1, "BatchNorm sums as fp64 atomic accumulators (1) instead of per-tile "
                  "partials combined by the consumer or a finalize launch (0)"),
    "fused_head": (1, "CIFAR head in one launch (final BN finalize .. final BN backward "
                      "sums) instead of eight"),
    "mat_bn_elems": (7000000, "inner bottleneck BN-ReLU materialized once (instead of applied in "
                              "the consumer's staging) up to this many elements ..."),
    "bap_maxc": (512, "identity bottleneck blocks whose input has <= this many channels run "
                         "their first 1x1 dgrad twice (sums, then BN backward + add in the "
                         "second pass; the streaming bn_dgrad1x1 kernel for K <= 256) instead "
                         "of dgrad + a separate BN-backward apply (RN50 bs128: 12.15 -> 11.67 "
                         "ms at 512 = stages 1-2; 11.87 at 1024: the K = 256 stage-3 pass "
                         "pair 110 vs 97 us unfused); 0 off"),
    "fwd1x1_stream": (1, "1x1 stride-1 forward convs whose weights fit in VGPRs (the "
                         "bottlenecks' expanding conv, the stage 1-2 narrowing conv and "
                         "projection) on the streaming kernel bn_fwd1x1 (BN prologue, "
                         "residual and BN statistics fused; 2x the implicit-GEMM tile's "
                         "bytes/s: RN50 11.69 -> 11.03 ms for the expanding convs)"),
    "dgrad1x1_stream": (1, "1x1 stride-1 dgrads carrying BN-backward sums whose weights fit "
                           "in VGPRs (the expanding conv at stages 1-2, the first conv at "
                           "stage 3) on the streaming kernel bn_dgrad1x1 (store + sums)"),
    "persist": (-1, "persistent small-batch CIFAR step (forward and backward each ONE launch, "
                    "one workgroup per image row slice; train/persist.py): -1 auto = per-rank "
                    "batch <= 240, 0 off, 1 whenever the network is supported"),
    "persist_slices": (-1, "row slices per image of the persistent step: -1 auto (backward: 4 "
                           "while 4N + 32 <= CUs, 2 while 2N + 64 <= CUs, else 1; forward: 4 "
                           "while 4N < 3/4 of the CUs, 2 while 2N + 16 <= CUs, else 1), 1, 2 "
                           "or 4 for both"),
    "persist_overlap": (1, "world > 1: the persistent step's first two stage buckets packed, "
                           "all-reduced and updated on the comm stream while the backward launch "
                           "runs (48 CUs left out of its grid), the last after it on the main "
                           "stream; 0: one pack + one all-reduce + one update after the backward "
                           "(profiles/cifar_comm_overlap.md)"),
    "opt_fused": (1, "the persistent step's optimizer as ONE launch (split-K slab sums on "
                     "one GPU, SGD-momentum, both bf16 weight copies: sgd_tiles) instead of "
                     "the grouped slab reduce + sgd_pack + ohwi_pack"),
    "mat_bn_minc": (256, "... and from this many channels (ImageNet stages 3-4: +1.3 %)"),
}


def overrides() -> dict:
    """The DTR_TUNE entries as {key: string value}."""
    out = {}
    for item in filter(None, os.environ.get("DTR_TUNE", "").split(",")):
        k, sep, v = item.partition("=")
        if not sep:
            raise ValueError(f"DTR_TUNE entry {item!r} is not key=value")
        out[k.strip()] = v.strip()
    return out


def validate(native_keys=()) -> None:
    """Every DTR_TUNE key must be an engine or a native tuning key."""
    native_keys = set(native_keys)
    known = set(ENGINE) | native_keys
    ov = overrides()
    bad = sorted(set(ov) - known)
    if bad:
        raise ValueError(f"unknown DTR_TUNE key(s) {bad}; known: {sorted(known)}")
    # native values are integers (csrc/tune.cpp rejects anything else); so are the
    # engine's integer keys -- a fractional value is an error, never truncated
    for k, v in ov.items():
        if k in native_keys or isinstance(ENGINE.get(k, (0.0,))[0], int):
            _int(k, v)


def _int(key: str, v: str) -> int:
    try:
        return int(v)
    except ValueError:
        raise ValueError(f"DTR_TUNE {key}={v!r}: an integer is required") from None


def get(key: str):
    """Current value of an engine key (its default's type)."""
    default = ENGINE[key][0]
    v = overrides().get(key)
    if v is None:
        return default
    return _int(key, v) if isinstance(default, int) else type(default)(v)
