"""One variant of scripts/comm_step_time.py for a rocprofv3 kernel trace:
    rocprofv3 --kernel-trace -d gpurun_out/prof_X -- python3 scripts/comm_step_trace.py MODE N STEPS
MODE: nocomm | ov0 (buckets after the backward) | ov1 (buckets overlapping it)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from comm_step_time import build  # noqa: E402


def main():
    mode, N, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    eng = build(N, mode != "nocomm", 1 if mode == "ov1" else 0)
    for _ in range(steps):
        eng.step()
    torch.cuda.synchronize()
    assert not eng.persist_error()
    print(mode, N, eng.plan.names(), flush=True)


if __name__ == "__main__":
    main()
