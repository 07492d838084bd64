#!/usr/bin/env python3
"""Diagnose fwd1x1_stream=0 vs 1 on a shallow bottleneck net: per-activation and
per-parameter-gradient relative differences after one forward + backward."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.models.params import ParamStore  # noqa: E402
from distributed_tensorflow_resnet_amd.models.spec import imagenet_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule  # noqa: E402


def run(mode):
    os.environ["DTR_TUNE"] = f"fwd1x1_stream={mode}"
    spec = imagenet_spec(0, image_hw=64, block="bottleneck", layers=[2, 2, 2, 2])
    gpu = torch.device("cuda", 0)
    eng = Engine(spec, 8, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(), device=gpu,
                 input_mode="nhwc", use_graph=False)
    torch.manual_seed(0)
    imgs = torch.randn(8, spec.image_h, spec.image_w, 3, device=gpu).to(torch.bfloat16).float()
    labels = torch.randint(0, spec.num_classes, (8,), device=gpu)
    eng.set_batch(imgs, labels)
    st = torch.cuda.current_stream().cuda_stream
    eng._run("fwd", st)
    torch.cuda.synchronize()
    acts = {f"X{i}": t.float().clone() for i, t in enumerate(eng.X)}
    bn = {n: (b.mean.clone(), b.rstd.clone(), b.scale.clone()) for n, b in eng.bns.items()}
    eng._run("bwd", st)
    if "gsum" in eng.seg:   # persistent step on one GPU: the slab sums
        eng._run("gsum", st)
    torch.cuda.synchronize()
    return spec, acts, bn, eng.grad.clone(), eng.scalars[0].item()


def rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


spec, a0, b0, g0, l0 = run("0")
_, a1, b1, g1, l1 = run("1")
print("loss", l0, l1)
for k in a0:
    print("act", k, f"{rel(a1[k], a0[k]):.2e}")
for n in b0:
    print("bn", n, " ".join(f"{rel(x1, x0):.2e}" for x0, x1 in zip(b0[n], b1[n])))
store = ParamStore(spec)
for sl in store.train_slots:
    d = rel(g1[sl.offset:sl.offset + sl.numel], g0[sl.offset:sl.offset + sl.numel])
    if d > 1e-3:
        print("grad", sl.name, f"{d:.2e}")
