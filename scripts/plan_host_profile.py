#!/usr/bin/env python3
"""Host issue time per plan op during real (unblocked) training steps.

A host call that blocks (e.g. a cross-stream wait on a busy GPU) shows up as an
op with a large host time; the main stream idles behind it once the host has
no queued work left.  Usage: plan_host_profile.py [batch] [model]"""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.models.spec import build_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    eng = Engine(build_spec("cifar10", 50), batch, weight_decay=2e-4,
                 lr_schedule=cifar_lr_schedule(), device=dev)
    eng.fill_synthetic(0)
    for _ in range(10):
        eng.step()
    torch.cuda.synchronize()
    K = 20
    eng.plan.set_profile(True)
    t0 = time.perf_counter()
    for _ in range(K):
        eng.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    eng.plan.set_profile(False)
    host = [h / K for h in eng.plan.host_us()]
    names = eng.plan.names()
    streams = eng.plan.op_streams()
    print(f"batch {batch}: host {1e3 * (t1 - t0) / K:.3f} ms/step issue, "
          f"{1e3 * (t2 - t0) / K:.3f} ms/step wall, plan ops {len(names)}, "
          f"sum op host {sum(host) / 1e3:.3f} ms")
    by = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for n, h in zip(names, host):
        e = by[n]
        e[0] += 1
        e[1] += h
        e[2] = max(e[2], h)
    print(f"{'op':28s} {'count':>5s} {'total us':>9s} {'mean us':>8s} {'max us':>8s}")
    for n, (c, tot, mx) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:28s} {c:5d} {tot:9.1f} {tot / c:8.2f} {mx:8.2f}")
    print("slowest ops:")
    for i in sorted(range(len(host)), key=lambda i: -host[i])[:25]:
        print(f"  #{i:4d} s{streams[i]} {names[i]:24s} {host[i]:8.2f} us")


if __name__ == "__main__":
    main()
