#!/usr/bin/env python3
"""Per-call main-stream timeline of one training step, labelled by layer.

Run 1 (under rocprofv3 --kernel-trace): builds the engine with the plan's conv_gemm
builder wrapped so every conv op records (mode, geometry, fusions), runs the step, and
dumps the labels of the plan's ops:
    rocprofv3 --kernel-trace -d gpurun_out/prof_calls -o run -- \\
        python3 scripts/step_calls.py --dump gpurun_out/calls.json [--model M --batch B]
Run 2 (anywhere): joins the last step's main-stream kernels, in order, to the plan's
main-stream launch ops and prints each call (duration, gap before it) and totals by label:
    python3 scripts/step_calls.py --report DB gpurun_out/calls.json > out.md
"""
import argparse
import collections
import json
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dump(a):
    import torch

    import distributed_tensorflow_resnet_amd as dtr
    from distributed_tensorflow_resnet_amd.models.spec import build_spec
    from distributed_tensorflow_resnet_amd.train.engine import (Engine, cifar_lr_schedule,
                                                                imagenet_lr_schedule)
    nat = dtr.native()
    labels = {}
    orig = nat.Plan.conv_gemm

    def conv_gemm(self, mode, a_, b_, out, out_f32, res, pre_s, pre_h, bias, nbias, stat,
                  accumulate, geom, bnb, *rest):
        N, H, W, C, K, kh, kw, s = geom[:8]
        tags = [t for t, on in (("pre", pre_s), ("stats", stat or rest[0]), ("res", res),
                                ("acc", accumulate), ("bnb", bnb)) if on]
        labels[self.size()] = (f"{'fwd' if mode == 0 else 'dgrad'} {H}x{W} {C}->{K} "
                               f"{kh}x{kw}/{s}" + (" +" + "+".join(tags) if tags else ""))
        return orig(self, mode, a_, b_, out, out_f32, res, pre_s, pre_h, bias, nbias, stat,
                    accumulate, geom, bnb, *rest)

    nat.Plan.conv_gemm = conv_gemm
    ds = "cifar10" if a.model.startswith("cifar") else "imagenet"
    size = int(a.model.rsplit("resnet", 1)[1])
    sched = cifar_lr_schedule() if ds == "cifar10" else imagenet_lr_schedule()
    eng = Engine(build_spec(ds, size), a.batch, weight_decay=1e-4, lr_schedule=sched,
                 device=torch.device("cuda", 0))
    eng.fill_synthetic(0)
    for _ in range(a.warmup + a.steps):
        eng.step()
    torch.cuda.synchronize()
    p = eng.plan
    ops = [{"name": n, "stream": s, "kind": k, "label": labels.get(i, n)}
           for i, (n, s, k) in enumerate(zip(p.names(), p.op_streams(), p.op_kinds()))]
    json.dump({"model": a.model, "batch": a.batch, "ops": ops}, open(a.dump, "w"))
    print(f"{len(ops)} plan ops, {sum(1 for o in ops if o['kind'] == 0)} launches")


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("dtr::", "")
    return n.split("<")[0][:40]


def report(a):
    meta = json.load(open(a.report[1]))
    ops = [o for o in meta["ops"] if o["kind"] == 0 and o["stream"] == 0]
    c = sqlite3.connect(a.report[0])
    rows = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    opt = [i for i, r in enumerate(rows) if "sgd_pack_kernel" in r[0]]
    main_sid = rows[opt[-1]][3]
    step = [r for r in rows[opt[-2] + 1:opt[-1] + 1] if r[3] == main_sid]
    print(f"# Main-stream calls of one {meta['model']} bs{meta['batch']} step (1x MI355X)\n")
    print(f"rocprofv3 --kernel-trace, last step; {len(step)} main-stream kernels, "
          f"{len(ops)} main-stream plan launches (`scripts/step_calls.py`).\n")
    # conv ops launch exactly one conv kernel each, in plan order: label conv kernels by
    # the plan's conv labels (rotated to start after the previous step's optimizer) and
    # every other kernel by its name (some plan ops launch nothing on some steps)
    k0 = max(i for i, o in enumerate(ops) if o["name"].startswith("sgd"))
    rot = ops[k0 + 1:] + ops[:k0 + 1]
    conv_labels = [o["label"] for o in rot if o["name"] == "conv_gemm"]
    conv_k = [r for r in step if "conv_gemm" in r[0] or "conv_ring" in r[0] or "direct" in r[0]]
    if len(conv_labels) != len(conv_k):
        print(f"(conv op / kernel counts differ: {len(conv_labels)} vs {len(conv_k)})\n")
    it = iter(conv_labels)
    seq = [{"label": next(it, short(r[0])) if r in conv_k else short(r[0])} for r in step]
    by = collections.defaultdict(lambda: [0, 0.0, 0.0])
    print("| # | call | kernel | us | gap before us |\n|---|---|---|---|---|")
    prev_end = None
    tot_k = tot_g = 0.0
    for i, (o, r) in enumerate(zip(seq, step)):
        dur = (r[2] - r[1]) / 1e3
        gap = (r[1] - prev_end) / 1e3 if prev_end is not None else 0.0
        prev_end = r[2]
        tot_k += dur
        tot_g += max(gap, 0.0)
        b = by[o["label"]]
        b[0] += 1
        b[1] += dur
        b[2] += max(gap, 0.0)
        print(f"| {i} | {o['label']} | `{short(r[0])}` | {dur:.1f} | {gap:.1f} |")
    print(f"\nMain stream: kernels {tot_k / 1e3:.3f} ms + gaps {tot_g / 1e3:.3f} ms = "
          f"{(step[-1][2] - step[0][1]) / 1e6:.3f} ms span.\n")
    print("| call | count | kernel ms | gap ms |\n|---|---|---|---|")
    for lab, (n, k, g) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        print(f"| {lab} | {n} | {k / 1e3:.3f} | {g / 1e3:.3f} |")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dump")
    ap.add_argument("--report", nargs=2)
    ap.add_argument("--model", default="imagenet_resnet50")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    if a.dump:
        dump(a)
    else:
        report(a)


if __name__ == "__main__":
    main()
