#!/usr/bin/env python3
"""Persistent multi-layer prototype (csrc/persist.hip) vs per-layer launches, CIFAR
ResNet-50 v2 stage 3 forward (3x3 64 -> 64 convs on 8x8 maps) at small batch.

For N images and L chained convs (the 16 of stage 3: 8 building blocks x 2):
  persistent  one launch, grid barriers between layers (2 workgroups per image)
  launches    L launches of the engine's own direct conv (BN+ReLU prologue, residual,
              BN-statistics epilogue), issued by the native plan executor back to back
Reports us per layer (median over rounds) and checks the prototype against a PyTorch
fp32 reference of the same chain (batch-statistics BN, bf16 rounding where the kernel
rounds).   python3 scripts/persist_probe.py [N ...]
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402

BF = torch.bfloat16
EPS = 1.001e-5


def make_inputs(N, L, dev, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x0 = torch.randn(N, 8, 8, 64, generator=g).to(dev).to(BF)
    bn0s = (torch.rand(64, generator=g) + 0.5).to(dev)
    bn0h = (torch.randn(64, generator=g) * 0.1).to(dev)
    w = (torch.randn(L, 64, 3, 3, 64, generator=g) / 24.0).to(dev).to(BF)
    gamma = (torch.rand(L, 64, generator=g) + 0.5).to(dev)
    beta = (torch.randn(L, 64, generator=g) * 0.1).to(dev)
    return x0, bn0s, bn0h, w, gamma, beta


def reference(x0, bn0s, bn0h, w, gamma, beta):
    L = w.shape[0]
    ys = []
    inp, sc, sh = x0.float(), bn0s, bn0h
    for layer in range(L):
        a = torch.relu(inp * sc + sh).to(BF).float()
        y = F.conv2d(a.permute(0, 3, 1, 2), w[layer].float().permute(0, 3, 1, 2), padding=1)
        y = y.permute(0, 2, 3, 1)
        if layer & 1:
            y = y + (x0 if layer == 1 else ys[layer - 2]).float()
        y = y.to(BF)
        ys.append(y)
        yf = y.float().reshape(-1, 64)
        mean = yf.mean(0)
        var = (yf * yf).mean(0) - mean * mean
        sc = gamma[layer] * torch.rsqrt(var + EPS)
        sh = beta[layer] - mean * sc
        inp = y.float()
    return torch.stack(ys)


def run_persistent(nat, x0, bn0s, bn0h, w, gamma, beta, reps=1):
    """reps back-to-back launches (own zeroed stats / barrier each); -> (y, us per launch)."""
    N, L = x0.shape[0], w.shape[0]
    dev = x0.device
    y = torch.empty(L, N, 8, 8, 64, device=dev, dtype=BF)
    stats = torch.zeros(reps, L * 2 * 64, device=dev)
    bar = torch.zeros(reps, 64, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for r in range(reps):
        nat.persist_stage_fwd(x0.data_ptr(), bn0s.data_ptr(), bn0h.data_ptr(), w.data_ptr(),
                              gamma.data_ptr(), beta.data_ptr(), y.data_ptr(),
                              stats[r].data_ptr(), bar[r].data_ptr(), err.data_ptr(), N, L, EPS,
                              st.cuda_stream)
    b.record()
    b.synchronize()
    if int(err.item()):
        raise RuntimeError("persist_stage_fwd: a grid barrier timed out")
    return y, a.elapsed_time(b) * 1e3 / reps


def run_launches(nat, x0, w, reps=1):
    """The same chain as L launches of the engine's direct conv from one native plan."""
    N, L = x0.shape[0], w.shape[0]
    dev = x0.device
    g = fn.ConvGeom(N, 8, 8, 64, 64, 3, 3, 1).as_list()
    ys = [torch.empty(N, 8, 8, 64, device=dev, dtype=BF) for _ in range(L)]
    sc, sh = torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev) * 0.1
    tiles, _ = fn.stat_tiles(N * 64, 64)
    part = torch.empty(tiles * 2 * 64, device=dev)
    plan = nat.Plan()
    for layer in range(L):
        src = x0 if layer == 0 else ys[layer - 1]
        res = 0
        if layer & 1:
            res = (x0 if layer == 1 else ys[layer - 2]).data_ptr()
        plan.conv_gemm(0, src.data_ptr(), w[layer].data_ptr(), ys[layer].data_ptr(), 0, res,
                       sc.data_ptr(), sh.data_ptr(), 0, 0, part.data_ptr(), 0, g,
                       [], [], [], [], [], 0.997, EPS, 1)
    st = torch.cuda.current_stream().cuda_stream
    plan.run(0, plan.size(), st, st)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        plan.run(0, plan.size(), st, st)
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    nat = fn.native()
    dev = torch.device("cuda")
    Ns = [int(v) for v in sys.argv[1:]] or [16, 32, 64]
    L = 16
    print("# Persistent multi-layer prototype vs per-layer launches (CIFAR RN50 stage 3 forward)\n")
    print(f"{L} chained 3x3 64->64 convs on 8x8 maps (BN+ReLU prologue, residual on every "
          "second, BN statistics), `scripts/persist_probe.py`; medians of 5 rounds x 20 "
          "back-to-back runs.\n")
    print("| images | workgroups | persistent us/layer | launches us/layer | ratio | "
          "max rel. err vs fp32 ref |\n|---|---|---|---|---|---|")
    for N in Ns:
        ins = make_inputs(N, L, dev)
        y, _ = run_persistent(nat, *ins)
        ref = reference(*ins)
        rel = max(((y[i].float() - ref[i].float()).norm() / ref[i].float().norm()).item()
                  for i in range(L))
        tp = statistics.median(run_persistent(nat, *ins, reps=20)[1] for _ in range(5)) / L
        tl = statistics.median(run_launches(nat, ins[0], ins[3], reps=20) for _ in range(5)) / L
        print(f"| {N} | {2 * N} | {tp:.2f} | {tl:.2f} | {tp / tl:.2f} | {rel:.2e} |", flush=True)


if __name__ == "__main__":
    main()
