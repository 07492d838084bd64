"""Timeline of one conv_ring8 workgroup (csrc/conv_ring8.hip, set_ring8_probe) and the
kernel time, for the RN50 3x3 shapes.  usage: python scripts/ring8_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributed_tensorflow_resnet_amd.ops.functional as fn  # noqa: E402

BF = torch.bfloat16
SHAPES = [("fwd", 128, 28, 128, 128, 3, 1), ("fwd", 128, 14, 256, 256, 3, 1),
          ("fwd", 128, 7, 512, 512, 3, 1), ("dgrad", 128, 14, 256, 256, 3, 1)]


def main():
    nat = fn.native()
    dev = torch.device("cuda", 0)
    for mode, N, H, C, K, k, s in SHAPES:
        g = fn.ConvGeom(N, H, H, C, K, k, k, s)
        if mode == "fwd":
            x = torch.randn(N, H, H, C, device=dev).to(BF)
            w = (torch.randn(K, k, k, C, device=dev) / 30).to(BF)
            run = lambda: fn.conv2d_fwd(x, w, s)  # noqa: E731
        else:
            dy = torch.randn(N, g.Ho, g.Wo, K, device=dev).to(BF)
            w = (torch.randn(k, k, C, K, device=dev) / 30).to(BF)
            run = lambda: fn.conv2d_dgrad(dy, w, (N, H, H, C), s)  # noqa: E731
        gflop = 2.0 * N * g.Ho * g.Wo * K * k * k * C / 1e9
        for r8 in (1, 0):
            nat.tune_set("ring8", r8)
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            print(f"{mode} N{N} {H}x{H} {C}->{K} k{k}s{s} ring8={r8}: {us:.1f} us, "
                  f"{gflop / us * 1e3:.0f} TF/s")
        nat.tune_set("ring8", 1)
        buf = torch.zeros(64, dtype=torch.int64, device=dev)
        nat.set_ring8_probe(buf.data_ptr())
        run()
        torch.cuda.synchronize()
        nat.set_ring8_probe(0)
        t = buf.cpu().tolist()
        if t[0]:
            base = t[0]
            tiles = [(v - base) / 100.0 for v in t[2:50] if v]
            steps = [b - a for a, b in zip([(t[1] - base) / 100.0] + tiles, tiles)]
            print(f"   WG0: prologue {(t[1] - base) / 100:.2f} us, {len(tiles)} K tiles: first "
                  f"{steps[:3]}, median {sorted(steps)[len(steps) // 2]:.2f} us/tile, loop end "
                  f"{(t[50] - base) / 100:.2f}, combine {(t[51] - t[50]) / 100:.2f}, epilogue "
                  f"{(t[52] - t[51]) / 100:.2f} us")


if __name__ == "__main__":
    main()
