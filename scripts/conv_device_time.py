#!/usr/bin/env python3
"""Device time per launch (incl. the ~1.5 us kernel boundary) of the CIFAR conv
kernels, from a native Plan of 200 back-to-back launches timed with HIP events:
direct fwd/dgrad/wgrad with each fusion toggled."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distributed_tensorflow_resnet_amd as dtr  # noqa: E402
from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402

BF = torch.bfloat16


def dev_time(plan, reps=3):
    st = torch.cuda.current_stream()
    best = 1e9
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        plan.run(0, plan.size(), st.cuda_stream, st.cuda_stream)
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / plan.size())
    return best


def main():
    nat = dtr.native()
    dev = torch.device("cuda", 0)
    n = 200
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    shapes = [(32, 16, 16, 3), (16, 32, 32, 3), (8, 64, 64, 3)]   # (H, C, K, k)
    if len(sys.argv) > 2 and sys.argv[2] == "imagenet":
        n = 20
        shapes = [(56, 64, 256, 1), (56, 64, 64, 3), (28, 128, 128, 3), (14, 256, 256, 3),
                  (28, 128, 512, 1), (7, 2048, 512, 1), (7, 512, 512, 3),
                  (14, 1024, 256, 1), (7, 512, 2048, 1)]
    for H, C, K, k in shapes:
        N = batch
        M = N * H * H
        g = fn.ConvGeom(N, H, H, C, K, k, k, 1).as_list()
        x = torch.randn(N, H, H, C, device=dev).to(BF)
        w = torch.randn(K, k, k, C, device=dev).to(BF)
        wh = w.permute(1, 2, 3, 0).contiguous()
        y = torch.empty(N, H, H, K, device=dev, dtype=BF)
        res = torch.randn_like(y)
        dxb = torch.empty_like(x)
        sc, sh = torch.rand(max(C, K), device=dev), torch.rand(max(C, K), device=dev)
        T = -(-M // nat.conv_gemm_bm(M, K))
        part = torch.empty(T * 2 * K, device=dev)
        Tb = -(-M // nat.conv_gemm_bm(M, C))
        bpart = torch.empty(Tb * 2 * C, device=dev)
        sp, pps = nat.wgrad_pick_splits(g)
        wpart = torch.empty(sp * k * k * C * K, device=dev)
        res_line = []
        variants = {
            "fwd": dict(pre=False, stats=False, res=False),
            "fwd+pre": dict(pre=True, stats=False, res=False),
            "fwd+stats": dict(pre=False, stats=True, res=False),
            "fwd+pre+stats+res": dict(pre=True, stats=True, res=True),
        }
        for name, v in variants.items():
            p = nat.Plan()
            for _ in range(n):
                p.conv_gemm(0, x.data_ptr(), w.data_ptr(), y.data_ptr(), 0,
                            res.data_ptr() if v["res"] else 0,
                            sc.data_ptr() if v["pre"] else 0, sh.data_ptr() if v["pre"] else 0,
                            0, 0, part.data_ptr() if v["stats"] else 0, 0, g, [], [], [], [], [],
                            0.997, 1e-5, 1)
            res_line.append(f"{name} {dev_time(p):.2f}")
        # consumer-side BN finalize in the prologue (BnPreFin) over `cnt` group partials
        if k == 3 and C == K and C <= 64:
            for cnt in (min(T, nat.pfin_cap(C)), 32, 8):
                gp = torch.rand(cnt * 2 * C, device=dev) + 0.1
                gam = torch.rand(C, device=dev)
                outs = [torch.empty(C, device=dev) for _ in range(6)]
                p = nat.Plan()
                for _ in range(n):
                    p.conv_gemm(0, x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, res.data_ptr(),
                                outs[2].data_ptr(), outs[3].data_ptr(), 0, 0, part.data_ptr(), 0,
                                g, [], [], [], [gp.data_ptr(), cnt, M // cnt, M, gam.data_ptr(),
                                               gam.data_ptr()] + [o.data_ptr() for o in outs],
                                [], 0.997, 1e-5, 1)
                res_line.append(f"fwd+pfin{cnt} {dev_time(p):.2f}")
        # dependency chain: every conv reads the previous conv's output (ping-pong)
        if C == K:
            y2 = torch.empty_like(y)
            p = nat.Plan()
            for i in range(n):
                src, dst = (y, y2) if i % 2 else (y2, y)
                p.conv_gemm(0, src.data_ptr(), w.data_ptr(), dst.data_ptr(), 0, res.data_ptr(),
                            sc.data_ptr(), sh.data_ptr(), 0, 0, part.data_ptr(), 0, g, [], [], [],
                            [], [], 0.997, 1e-5, 1)
            y2.copy_(x)
            res_line.append(f"chain(fwd+pre+stats+res) {dev_time(p):.2f}")
            # chain over 16 distinct activation / partial buffers (like the real forward)
            bufs = [torch.randn_like(x) for _ in range(17)]
            parts = [torch.empty_like(part) for _ in range(16)]
            p = nat.Plan()
            for i in range(n):
                j = i % 16
                p.conv_gemm(0, bufs[j].data_ptr(), w.data_ptr(), bufs[j + 1].data_ptr(), 0,
                            bufs[(j + 5) % 17].data_ptr(), sc.data_ptr(), sh.data_ptr(), 0, 0,
                            parts[j].data_ptr(), 0, g, [], [], [], [], [], 0.997, 1e-5, 1)
            res_line.append(f"chain16bufs {dev_time(p):.2f}")
            del bufs, parts
        for name, bnb in (("dgrad", False), ("dgrad+bnb", True)):
            p = nat.Plan()
            bl = [x.data_ptr(), sc.data_ptr(), sh.data_ptr(), sc.data_ptr(), sh.data_ptr(),
                  bpart.data_ptr()] if bnb else []
            for _ in range(n):
                p.conv_gemm(1, res.data_ptr(), wh.data_ptr(), dxb.data_ptr(), 0, 0, 0, 0, 0, 0, 0,
                            0, g, bl, [], [], [], [], 0.997, 1e-5, 1)
            res_line.append(f"{name} {dev_time(p):.2f}")
        for name, pre in (("wgrad", False), ("wgrad+pre", True)):
            p = nat.Plan()
            for _ in range(n):
                p.conv_wgrad(res.data_ptr(), x.data_ptr(), sc.data_ptr() if pre else 0,
                             sh.data_ptr() if pre else 0, wpart.data_ptr(), g, sp, pps)
            res_line.append(f"{name} {dev_time(p):.2f}")
        p = nat.Plan()
        for _ in range(n):
            p.fill(sc.data_ptr(), C, 1.0)
        res_line.append(f"fill {dev_time(p):.2f}")
        flop = 2.0 * M * K * k * k * C
        print(f"N={N} H={H} C={C} K={K} k={k} ({flop / 1e9:.1f} GF; us/launch): " +
              " | ".join(res_line), flush=True)


if __name__ == "__main__":
    main()
