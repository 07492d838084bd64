#!/usr/bin/env python3
"""Compare the engine with BN accumulator mode on/off (tune bn_acc): per-BN forward
statistics after the forward segment, per-tensor gradients after the backward."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.models.spec import cifar_spec, imagenet_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule  # noqa: E402


def run(acc, size, N):
    os.environ["DTR_TUNE"] = f"bn_acc={acc}"
    spec = cifar_spec(size) if size < 0 or size % 6 == 2 else imagenet_spec(size, image_hw=64)
    dev = torch.device("cuda", 0)
    eng = Engine(spec, N, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(), device=dev,
                 input_mode="nhwc", use_graph=False)
    torch.manual_seed(0)
    imgs = torch.randn(N, spec.image_h, spec.image_w, 3, device=dev).to(torch.bfloat16).float()
    labels = torch.randint(0, spec.num_classes, (N,), device=dev)
    eng.set_batch(imgs, labels)
    st = torch.cuda.current_stream().cuda_stream
    eng._run("fwd", st)
    torch.cuda.synchronize()
    stats = {n: (b.mean.clone(), b.rstd.clone()) for n, b in eng.bns.items()}
    eng._run("bwd", st)
    if "gsum" in eng.seg:   # persistent step on one GPU: the slab sums
        eng._run("gsum", st)
    torch.cuda.synchronize()
    grads = {s.name: eng.grad[s.offset:s.offset + s.numel].clone() for s in eng.params.train_slots}
    return stats, grads, eng.scalars[0].item()


def rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-20)).item()


size = int(sys.argv[1]) if len(sys.argv) > 1 else 20
N = int(sys.argv[2]) if len(sys.argv) > 2 else 32
s0, g0, l0 = run("0", size, N)
for m in ("0", "1", "fwd", "bwd"):
    s1, g1, l1 = run(m, size, N)
    gs = sorted(((rel(g1[n], g0[n]), n) for n in g0), reverse=True)[:3]
    tot = rel(torch.cat([g1[n] for n in g0]), torch.cat([g0[n] for n in g0]))
    print(f"mode {m}: loss {l1:.5f} vs {l0:.5f}; global grad rel {tot:.2e}; worst {gs}")
s1, g1, l1 = run("fwd", size, N)
for n in s0:
    print(f"BN {n:32s} mean {rel(s1[n][0], s0[n][0]):.2e} rstd {rel(s1[n][1], s0[n][1]):.2e}")
