#!/usr/bin/env python3
"""Per-layer roofline of the ImageNet ResNet-50 v2 convolutions at 128 images (1x MI355X).

For every conv shape of the step (with the step's fusions: forward
with the BN+ReLU prologue and BN-statistics epilogue into fp64 accumulators, dgrad with
the next BN-backward sums, split-K wgrad with the BN+ReLU prologue plus its reduce),
times the kernels with HIP events (median of `reps`) and prints, per pass:

  FLOP, unique bytes (each operand read once, each output written once), the floor
  max(FLOP / 2.3 PF/s, bytes / 5 TB/s), achieved us, achieved / floor, and the step
  share (x layers of that shape).

    python3 scripts/roofline.py [reps] > profiles/imagenet_resnet50_roofline.md
Run under rocprofv3 --pmc FETCH_SIZE ... for the measured bytes of each kernel.
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402
from distributed_tensorflow_resnet_amd.utils import tune  # noqa: E402

PEAK_FLOPS = 2.3e15   # dense bf16 MFMA, sustained (2.5 PF/s headline, no sparsity)
PEAK_BYTES = 5.0e12   # HBM3E, achievable streaming

# (H_in, Cin, Cout, k, s, layers per step) -- ImageNet RN50 v2
SHAPES = [
    (56, 64, 256, 1, 1, 4), (56, 64, 64, 1, 1, 1), (56, 64, 64, 3, 1, 3), (56, 256, 64, 1, 1, 2),
    (56, 256, 128, 1, 1, 1), (56, 128, 128, 3, 2, 1), (56, 256, 512, 1, 2, 1),
    (28, 128, 512, 1, 1, 4), (28, 128, 128, 3, 1, 3), (28, 512, 128, 1, 1, 3),
    (28, 512, 256, 1, 1, 1), (28, 256, 256, 3, 2, 1), (28, 512, 1024, 1, 2, 1),
    (14, 256, 1024, 1, 1, 6), (14, 256, 256, 3, 1, 5), (14, 1024, 256, 1, 1, 5),
    (14, 1024, 512, 1, 1, 1), (14, 512, 512, 3, 2, 1), (14, 1024, 2048, 1, 2, 1),
    (7, 512, 2048, 1, 1, 3), (7, 512, 512, 3, 1, 2), (7, 2048, 512, 1, 1, 2),
]


def timed(fnc, reps):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fnc()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def set_cfg(nat, cfg):
    """Apply 'key=v,key=v' native tuning entries (in-process A/B)."""
    for item in filter(None, cfg.split(",")):
        k, v = item.split("=")
        nat.tune_set(k, int(v))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    # --ab CFG_A CFG_B ...: time every pass under each native tuning config in turn, in
    # one process (run-to-run clock drift between processes reached 10-25 %)
    ab = sys.argv[sys.argv.index("--ab") + 1:] if "--ab" in sys.argv else []
    # under rocprofv3 --pmc: write the (layer, pass) of every call in launch order, so
    # scripts/pmc_roofline.py can attribute the per-dispatch counters
    manifest = open(os.environ["ROOFLINE_MANIFEST"], "w") if os.environ.get("ROOFLINE_MANIFEST") else None
    N = int(os.environ.get("ROOFLINE_N", "128"))
    dev = torch.device("cuda")
    BF = torch.bfloat16
    nat = fn.native()
    rows = []
    ab_rows = []
    tot = {"fwd": [0.0, 0.0], "dgrad": [0.0, 0.0], "wgrad": [0.0, 0.0]}
    for H, C, K, k, s, cnt in SHAPES:
        g = fn.ConvGeom(N, H, H, C, K, k, k, s)
        Ho = g.Ho
        x = torch.randn(N, H, H, C, device=dev).to(BF)
        w = (torch.randn(K, k, k, C, device=dev) * 0.05).to(BF)
        whwio = w.permute(1, 2, 3, 0).contiguous()
        sc = torch.rand(C, device=dev) + 0.5
        sh = torch.randn(C, device=dev) * 0.1
        dy = torch.randn(N, Ho, Ho, K, device=dev).to(BF)
        M = N * Ho * Ho
        tiles, _ = fn.stat_tiles(M, K)
        part = torch.empty(tiles * 2 * K, device=dev)
        acc = torch.zeros(8 * 2 * K, device=dev, dtype=torch.float64)
        out = torch.empty(N, Ho, Ho, K, device=dev, dtype=BF)
        dx = torch.empty_like(x)
        Mx = N * H * H
        bnb = (x, torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5, sc, sh,
               torch.zeros((Mx // 64 + 1) * 2 * C, device=dev))
        bacc = torch.zeros(8 * 2 * C, device=dev, dtype=torch.float64)
        gw = torch.empty(k, k, C, K, device=dev)
        flop = 2.0 * M * K * k * k * C
        xb, yb, wb = N * H * H * C * 2, M * K * 2, K * k * k * C * 2
        sp, _ = nat.wgrad_pick_splits(g.as_list())
        slab = sp * K * k * k * C * 4
        # the engine applies the input BN+ReLU in the conv (PRE) unless it materializes
        # it (train/engine.py _materialize_bn: stages 3-4)
        pre = dict(pre_scale=sc, pre_shift=sh)
        if C >= tune.get("mat_bn_minc") and N * H * H * C <= tune.get("mat_bn_elems"):
            pre = {}
        passes = {
            "fwd": (lambda: fn.conv2d_fwd(x, w, s, stat_part=part, out=out, fin=[acc], **pre),
                    xb + wb + yb),
            "dgrad": (lambda: fn.conv2d_dgrad(dy, whwio, tuple(x.shape), s, out=dx, bnb=bnb,
                                              bfin=[bacc]),
                      yb + wb + 2 * xb),
            "wgrad": (lambda: fn.conv2d_wgrad(dy, x, k, k, s, grad_hwio=gw, **pre),
                      yb + xb + 2 * slab + K * k * k * C * 4),
        }
        for p, (f, byts) in passes.items():
            if p == "dgrad" and C < 64:
                continue
            name = f"{H}x{H} {C}->{K} {k}x{k}/{s}" + (" PRE" if p != "dgrad" and pre else "")
            if manifest:
                manifest.write(f"{name}|{p}|{reps + 1}|{byts}|{flop}\n")
                manifest.flush()
            if ab:
                dflt = {t[0]: t[3] for t in nat.tune_table()}
                alts = []
                for rnd in range(3):
                    for i, cfg in enumerate(ab):
                        set_cfg(nat, cfg)
                        f()
                        torch.cuda.synchronize()
                        t_us = timed(f, reps)
                        if rnd == 0:
                            alts.append([])
                        alts[i].append(t_us)
                        set_cfg(nat, ",".join(f"{k}={v}" for k, v in dflt.items()))
                ab_rows.append((name, p, cnt, [statistics.median(a) for a in alts]))
                continue
            f()
            torch.cuda.synchronize()
            us = timed(f, reps)
            floor = max(flop / PEAK_FLOPS, byts / PEAK_BYTES) * 1e6
            rows.append((name, p, cnt, flop, byts, floor, us))
            tot[p][0] += cnt * floor
            tot[p][1] += cnt * us
        del x, w, whwio, dy, out, dx, bnb, gw, part
        torch.cuda.empty_cache()
    if ab:
        print(f"# In-process A/B, N = {N}: us per call (median of 3 alternating rounds x {reps})\n")
        print("| layer | pass | x/step | " + " | ".join(ab) + " |")
        print("|---|---|---|" + "---|" * len(ab))
        sums = [0.0] * len(ab)
        for name, p, cnt, ts in ab_rows:
            print(f"| {name} | {p} | {cnt} | " + " | ".join(f"{t:.1f}" for t in ts) + " |")
            for i, t in enumerate(ts):
                sums[i] += cnt * t
        print()
        for p in ("fwd", "dgrad", "wgrad"):
            per = [sum(cnt * ts[i] for name, pp, cnt, ts in ab_rows if pp == p) for i in range(len(ab))]
            print(f"- {p}: " + ", ".join(f"{c}: {v / 1e3:.3f} ms/step" for c, v in zip(ab, per)))
        return
    print(f"# ImageNet ResNet-50 v2 conv roofline, N = {N}, 1x MI355X\n")
    print("Floor = max(FLOP / 2.3 PF/s, unique bytes / 5 TB/s); unique bytes count each operand "
          "once (dgrad: dy, W, dx and the BN input x its epilogue reads; wgrad: dy, x, the fp32 "
          "split-K slabs written and read back, dW).  Forward and weight-gradient convs take "
          "the BN+ReLU prologue on their input (PRE) where the engine does.  `scripts/roofline.py`, HIP-event medians.\n")
    print("| layer | pass | x/step | GFLOP | MB | floor us | achieved us | x floor | TF/s | TB/s |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for name, p, cnt, flop, byts, floor, us in rows:
        print(f"| {name} | {p} | {cnt} | {flop / 1e9:.1f} | {byts / 1e6:.0f} | {floor:.1f} | "
              f"{us:.1f} | {us / floor:.2f} | {flop / us / 1e6:.0f} | {byts / us / 1e6:.2f} |")
    print()
    for p, (fl, us) in tot.items():
        print(f"- {p}: floor {fl / 1e3:.2f} ms/step, achieved {us / 1e3:.2f} ms/step "
              f"({us / max(fl, 1e-9):.2f}x)")


if __name__ == "__main__":
    main()
