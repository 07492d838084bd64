#!/usr/bin/env python3
"""Per-shape timing of the conv kernels on SURVEY Appendix-A shapes.

Prints one line per (shape, pass) with time and achieved TFLOP/s, and writes a
JSON summary to gpurun_out/kernels.json.  Random bf16 operands (DVFS-honest)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402

# (name, N, H, C, K, k, s)
SHAPES = [
    ("cifar_16x16_3x3", 128, 32, 16, 16, 3, 1),
    ("cifar_32x32_3x3", 128, 16, 32, 32, 3, 1),
    ("cifar_64x64_3x3", 128, 8, 64, 64, 3, 1),
    ("in_stem_7x7s2", 128, 224, 8, 64, 7, 2),
    ("in_56_64_256_1x1", 128, 56, 64, 256, 1, 1),
    ("in_56_64_64_3x3", 128, 56, 64, 64, 3, 1),
    ("in_56_256_64_1x1", 128, 56, 256, 64, 1, 1),
    ("in_28_128_128_3x3", 128, 28, 128, 128, 3, 1),
    ("in_28_512_128_1x1", 128, 28, 512, 128, 1, 1),
    ("in_28_128_512_1x1", 128, 28, 128, 512, 1, 1),
    ("in_14_256_256_3x3", 128, 14, 256, 256, 3, 1),
    ("in_14_1024_256_1x1", 128, 14, 1024, 256, 1, 1),
    ("in_14_256_1024_1x1", 128, 14, 256, 1024, 1, 1),
    ("in_7_512_512_3x3", 128, 7, 512, 512, 3, 1),
    ("in_7_2048_512_1x1", 128, 7, 2048, 512, 1, 1),
    ("in_7_512_2048_1x1", 128, 7, 512, 2048, 1, 1),
]


def timeit(f, iters=20):
    for _ in range(3):
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    dev = torch.device("cuda")
    only = sys.argv[1:] or None
    res = []
    for name, N, H, C, K, k, s in SHAPES:
        if only and not any(o in name for o in only):
            continue
        g = fn.ConvGeom(N, H, H, C, K, k, k, s)
        x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(K, k, k, C, device=dev) * 0.05).to(torch.bfloat16)
        whwio = w.permute(1, 2, 3, 0).contiguous()
        sc = torch.rand(C, device=dev) + 0.5
        sh = torch.randn(C, device=dev) * 0.1
        dy = torch.randn(N, g.Ho, g.Wo, K, device=dev).to(torch.bfloat16)
        flops = 2.0 * N * g.Ho * g.Wo * K * k * k * C
        tiles, _ = fn.stat_tiles(N * g.Ho * g.Wo, K)
        part = torch.empty(tiles * 2 * K, device=dev)
        out = torch.empty(N, g.Ho, g.Wo, K, device=dev, dtype=torch.bfloat16)
        dx = torch.empty_like(x)
        pre = dict(pre_scale=sc, pre_shift=sh) if C >= 16 else {}
        t_f = timeit(lambda: fn.conv2d_fwd(x, w, s, stat_part=part, out=out, **pre))
        t_d = timeit(lambda: fn.conv2d_dgrad(dy, whwio, tuple(x.shape), s, out=dx)) if C >= 16 else 0
        gw = torch.empty(k, k, C, K, device=dev)
        t_w = timeit(lambda: fn.conv2d_wgrad(dy, x, k, k, s, grad_hwio=gw, **pre))
        # roofline floor: bf16 x, w read once, y written once (5 TB/s), 1.3 PF/s bf16 MFMA
        nbytes = 2.0 * (x.numel() + w.numel() + out.numel())
        floor = max(nbytes / 5e12, flops / 1.3e15) * 1e6
        t_lib = 0.0
        if k == 1 and s == 1:   # plain GEMM of the same shape through hipBLASLt (library reference)
            x2, w2 = x.view(-1, C), w.view(K, C).t()
            t_lib = timeit(lambda: torch.mm(x2, w2, out=out.view(-1, K)))
        r = {"name": name, "gflop": flops / 1e9, "fwd_us": t_f, "dgrad_us": t_d, "wgrad_us": t_w,
             "floor_us": floor, "hipblaslt_us": t_lib,
             "fwd_tf": flops / t_f / 1e6, "dgrad_tf": flops / t_d / 1e6 if t_d else 0,
             "wgrad_tf": flops / t_w / 1e6}
        res.append(r)
        print(f"{name:22s} {flops/1e9:7.2f} GF | fwd {t_f:8.1f}us {r['fwd_tf']:6.1f}TF | "
              f"dgrad {t_d:8.1f}us {r['dgrad_tf']:6.1f}TF | wgrad {t_w:8.1f}us {r['wgrad_tf']:6.1f}TF"
              f" | floor {floor:7.1f}us | hipblaslt-mm {t_lib:7.1f}us",
              flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/kernels.json", "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
