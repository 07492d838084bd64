"""tfprof-style model analysis (resnet_single.py:58-66 used
tf.contrib.tfprof.model_analyzer for trainable-parameter and FLOP counts).

Computed from the static ModelSpec: per-layer parameter counts and
multiply-add FLOPs (2 x MAC) for forward; training ~= 3x forward (fwd + dgrad
+ wgrad)."""
from __future__ import annotations

from ..models.spec import ModelSpec


def conv_flops(c, batch: int) -> int:
    return 2 * batch * c.ho * c.wo * c.cout * c.kh * c.kw * c.cin


def analyze(spec: ModelSpec, batch: int = 1) -> dict:
    rows = []
    for c in spec.all_convs():
        rows.append({"name": c.name, "shape": c.shape, "params": c.kh * c.kw * c.cin * c.cout,
                     "flops": conv_flops(c, batch), "out": (c.ho, c.wo, c.cout)})
    dense_params = spec.dense_in * spec.num_classes + spec.num_classes
    rows.append({"name": "dense", "shape": (spec.dense_in, spec.num_classes),
                 "params": dense_params, "flops": 2 * batch * spec.dense_in * spec.num_classes,
                 "out": (spec.num_classes,)})
    bn_params = sum(2 * p.shape[0] for p in spec.params if p.kind == "gamma")
    fwd = sum(r["flops"] for r in rows)
    return {"layers": rows, "trainable_params": spec.num_trainable(), "bn_params": bn_params,
            "forward_flops": fwd, "train_flops": 3 * fwd, "batch": batch}


def report(spec: ModelSpec, batch: int = 1) -> str:
    a = analyze(spec, batch)
    lines = [f"{'layer':14s} {'kernel (HWIO)':22s} {'params':>10s} {'GFLOP':>10s}"]
    for r in a["layers"]:
        lines.append(f"{r['name']:14s} {str(r['shape']):22s} {r['params']:>10d} "
                     f"{r['flops'] / 1e9:>10.3f}")
    lines.append(f"total trainable params: {a['trainable_params']:,} "
                 f"(BN gamma/beta {a['bn_params']:,})")
    lines.append(f"forward GFLOP (batch {batch}): {a['forward_flops'] / 1e9:.2f}; "
                 f"train step ~{a['train_flops'] / 1e9:.2f}")
    return "\n".join(lines)
