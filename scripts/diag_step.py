#!/usr/bin/env python3
"""Phase timing (HIP events) of the CIFAR training step: forward, backward,
optimizer -- averaged over 100 steps.  Combine with DTR_DIAG_SKIP / DTR_TUNE=fork_wgrad=0
to find the critical path (timing only: skipped launches make the math wrong)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.models.spec import build_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule  # noqa: E402


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    eng = Engine(build_spec("cifar10", 50), batch, weight_decay=2e-4,
                 lr_schedule=cifar_lr_schedule(), device=torch.device("cuda", 0))
    eng.fill_synthetic(0)
    for _ in range(10):
        eng.step()
    acc = {}
    n = 100
    for _ in range(n):
        for k, v in eng.step_timed().items():
            acc[k] = acc.get(k, 0.0) + v / n
    tag = f"skip={os.environ.get('DTR_DIAG_SKIP', '')} fork={eng.fork_wgrad} batch={batch}"
    print(tag + " " + " ".join(f"{k}={v:.3f}ms" for k, v in acc.items()) +
          f" total={sum(acc.values()):.3f}ms", flush=True)


if __name__ == "__main__":
    main()
