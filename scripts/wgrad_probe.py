#!/usr/bin/env python3
"""Run one weight-gradient shape repeatedly (for rocprofv3 --pmc passes).
python3 scripts/wgrad_probe.py N H C K k s [reps] [ring 0|1]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402

N, H, C, K, k, s = (int(v) for v in sys.argv[1:7])
reps = int(sys.argv[7]) if len(sys.argv) > 7 else 20
nat = fn.native()
if len(sys.argv) > 8:
    nat.tune_set("ring_wgrad", int(sys.argv[8]))
BF = torch.bfloat16
x = torch.randn(N, H, H, C, device="cuda").to(BF)
g = fn.ConvGeom(N, H, H, C, K, k, k, s)
dy = torch.randn(N, g.Ho, g.Wo, K, device="cuda").to(BF)
gw = torch.empty(k, k, C, K, device="cuda")
for _ in range(reps):
    fn.conv2d_wgrad(dy, x, k, k, s, grad_hwio=gw)
torch.cuda.synchronize()
print("splits", nat.wgrad_pick_splits(g.as_list()))
