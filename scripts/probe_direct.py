#!/usr/bin/env python3
"""Inside-the-kernel timeline of the direct 3x3 conv (conv_direct.hip) on the CIFAR
shapes: every workgroup stamps wall_clock64 (100 MHz) at start, operands staged in
LDS, MFMAs done, and inside the epilogue (conv_epilogue.h) after the fp32 tile is
staged in LDS, after the row pass (residual / rounding / BN sums), after the
column-sum reductions (after the row stores are issued) and when the atomics are issued.  For a back-to-back chain of identical
launches (the step's pattern) this prints, per launch, the dispatch gap (previous
launch's last stamp -> this launch's first start), the start skew across
workgroups, and the median per-workgroup phase durations.

  python scripts/probe_direct.py [batch] [variant ...]   variants: fwd dgrad
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distributed_tensorflow_resnet_amd as dtr  # noqa: E402
from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402

BF = torch.bfloat16
SHAPES = [(32, 16), (16, 32), (8, 64)]
if os.environ.get("PROBE_SHAPES"):   # e.g. "56x64" (with DTR_TUNE=direct_wide=1)
    SHAPES = [tuple(int(v) for v in t.split("x")) for t in os.environ["PROBE_SHAPES"].split(",")]
NL = 6   # launches per chain


def main():
    nat = dtr.native(required=True)
    dev = torch.device("cuda", 0)
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    variants = sys.argv[2:] or ["fwd", "dgrad"]
    for H, C in SHAPES:
        N, K = batch, C
        gl = fn.ConvGeom(N, H, H, C, K, 3, 3, 1).as_list()
        M = N * H * H
        x = torch.randn(N, H, H, C, device=dev).to(BF)
        w = (torch.randn(K, 3, 3, C, device=dev) * 0.05).to(BF)
        wh = w.permute(1, 2, 3, 0).contiguous()
        y = torch.empty(N, H, H, K, device=dev, dtype=BF)
        res = torch.randn_like(y)
        dx, aout = torch.empty_like(x), torch.empty_like(x)
        V = [(torch.rand(C, device=dev) + 0.5) for _ in range(16)]
        P = [v.data_ptr() for v in V]
        rep = nat.bn_acc_rep()
        acc = torch.zeros(rep * 2 * max(C, K), dtype=torch.float64, device=dev)
        pacc = torch.rand(rep * 2 * C, dtype=torch.float64, device=dev) + M
        T = -(-M // nat.conv_gemm_bm(M, K))
        part = torch.empty(T * 2 * K, device=dev)
        bpart = torch.empty(T * 2 * C, device=dev)
        pfin_acc = [pacc.data_ptr(), 0xFFFFFFFF, M // T, M] + P[0:8]
        abwd_acc = [x.data_ptr(), res.data_ptr()] + P[8:13] + [pacc.data_ptr(), 0xFFFFFFFF,
                                                              aout.data_ptr(), P[13], P[14],
                                                              torch.empty(3 * C, device=dev).data_ptr()]
        bnb = [x.data_ptr(), P[2], P[3], P[4], P[5], bpart.data_ptr()]
        for var in variants:
            plan = nat.Plan()
            for _ in range(NL):
                if var == "fwd":   # the step's forward conv: BN-ReLU prologue from the
                    plan.conv_gemm(0, x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, res.data_ptr(),
                                   P[4], P[5], 0, 0, part.data_ptr(), 0, gl, [], [acc.data_ptr()],
                                   [], pfin_acc, [], 0.997, 1e-5, 1)   # accumulators, stats out
                else:              # the step's dgrad: BN-backward prologue, BN-backward sums out
                    plan.conv_gemm(1, res.data_ptr(), wh.data_ptr(), dx.data_ptr(), 0, 0, 0, 0, 0,
                                   0, 0, 0, gl, bnb, [], [acc.data_ptr()], [], abwd_acc, 0.997,
                                   1e-5, 1)
            # grid size: from a probe-less dry run count is not exposed; allocate generously
            probe = torch.zeros(NL * 8 * 8192, dtype=torch.int64, device=dev)
            st = torch.cuda.current_stream().cuda_stream
            for rnd in range(3):
                probe.zero_()
                nat.set_direct_probe(probe.data_ptr())
                plan.run(0, plan.size(), st, st, st)
                nat.set_direct_probe(0)
                torch.cuda.synchronize()
            pr = probe.view(-1, 8).cpu()
            rows = pr[pr[:, 0] != 0]
            nwg = rows.shape[0] // NL
            L = rows.view(NL, nwg, 8).double() * 10.0   # 100 MHz ticks -> ns
            t0 = L[:, :, 0].min()
            lines = []
            for i in range(1, NL):
                prev_end = L[i - 1, :, 3].max()
                start = L[i, :, 0]
                gap = (start.min() - prev_end) / 1e3
                skew = (start.max() - start.min()) / 1e3
                d = lambda a, b: statistics.median((L[i, :, b] - L[i, :, a]).tolist()) / 1e3  # noqa
                ph = [d(0, 1), d(1, 2), d(2, 4), d(4, 5), d(5, 6), d(6, 3)]
                span = (L[i, :, 3].max() - start.min()) / 1e3
                lines.append((gap, skew, *ph, span))
            med = [statistics.median(c) for c in zip(*lines)]
            print(f"N{N} H{H:2d} C{C:2d} {var:5s} wg {nwg:4d}: gap {med[0]:4.2f} | skew "
                  f"{med[1]:4.2f} | stage {med[2]:4.2f} | mfma {med[3]:4.2f} | epi: lds "
                  f"{med[4]:4.2f} rows+stores {med[5]:4.2f} colsum {med[6]:4.2f} atomics "
                  f"{med[7]:4.2f} | span {med[8]:5.2f} us", flush=True)


if __name__ == "__main__":
    main()
