#!/usr/bin/env python3
"""Pure host cost of issuing one training step: block the stream behind a long
sleep kernel, issue K steps, time the issue (must finish before the sleep)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_tensorflow_resnet_amd.models.spec import build_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for batch in (128, 32):
        for fork in ("1", "0"):
            os.environ["DTR_TUNE"] = f"fork_wgrad={fork}"
            eng = Engine(build_spec("cifar10", 50), batch, weight_decay=2e-4,
                         lr_schedule=cifar_lr_schedule(), device=dev)
            eng.fill_synthetic(0)
            for _ in range(5):
                eng.step()
            torch.cuda.synchronize()
            for k in (5, 20):
                torch.cuda._sleep(2_000_000_000)      # ~1 s of device time on the stream
                if eng.fork_wgrad:
                    eng.side.wait_stream(torch.cuda.current_stream())
                t0 = time.perf_counter()
                for _ in range(k):
                    eng.step()
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                print(f"batch {batch} fork={eng.fork_wgrad} K={k}: host issue "
                      f"{(t1 - t0) / k * 1e3:.3f} ms/step ({eng.plan.size()} plan ops)", flush=True)
            del eng
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
