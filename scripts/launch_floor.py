#!/usr/bin/env python3
"""Launch floor of the static plan on this runtime: what one kernel launch costs
the host, whether two host threads issuing to two streams scale, and what a
hipGraph replay of the same launches costs per node.

  python scripts/launch_floor.py [n_launches]
"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import distributed_tensorflow_resnet_amd as dtr  # noqa: E402


def timed(fn, reps=7):
    best_h, best_w = 1e9, 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        best_h, best_w = min(best_h, t1 - t0), min(best_w, t2 - t0)
    return best_h * 1e6, best_w * 1e6


def main():
    nat = dtr.native(required=True)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    bufs = [torch.zeros(1024, device=dev) for _ in range(2)]
    plans = []
    for b in bufs:
        p = nat.Plan()
        for _ in range(n):
            p.fill(b.data_ptr(), 1024, 1.0)
        plans.append(p)
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
    h, w = timed(lambda: plans[0].run(0, n, s0.cuda_stream, 0))
    print(f"1 thread, 1 stream, {n} fills: host {h / n:.2f} us/launch, wall {w / n:.2f} us/launch",
          flush=True)

    def both_serial():
        plans[0].run(0, n, s0.cuda_stream, 0)
        plans[1].run(0, n, s1.cuda_stream, 0)
    h, w = timed(both_serial)
    print(f"1 thread, 2 streams, 2x{n} fills: host {h / (2 * n):.2f} us/launch, "
          f"wall {w / (2 * n):.2f}", flush=True)

    def both_threads():
        t = threading.Thread(target=plans[1].run, args=(0, n, s1.cuda_stream, 0))
        t.start()
        plans[0].run(0, n, s0.cuda_stream, 0)
        t.join()
    h, w = timed(both_threads)
    print(f"2 threads, 2 streams, 2x{n} fills: host {h / (2 * n):.2f} us/launch (aggregate), "
          f"wall {w / (2 * n):.2f}", flush=True)

    # event record/wait pair cost
    pe = nat.Plan()
    for _ in range(n // 2):
        e = pe.new_event()
        pe.use_stream(0)
        pe.record(e)
        pe.use_stream(1)
        pe.wait(e)
        pe.fill(bufs[1].data_ptr(), 1024, 1.0)
        pe.use_stream(0)
        pe.fill(bufs[0].data_ptr(), 1024, 1.0)
    h, w = timed(lambda: pe.run(0, pe.size(), s0.cuda_stream, s1.cuda_stream))
    print(f"fork per launch pair ({n // 2} record+wait+2 fills): host {h / (n // 2):.2f} us/pair, "
          f"wall {w / (n // 2):.2f}", flush=True)

    # hipGraph replay of the same n fills (single stream)
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream()
    with torch.cuda.stream(cs):
        plans[0].run(0, n, cs.cuda_stream, 0)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=cs):
        plans[0].run(0, n, cs.cuda_stream, 0)
    h, w = timed(g.replay)
    print(f"hipGraph replay of {n} fills: host {h:.1f} us/replay, wall {w / n:.2f} us/node",
          flush=True)


if __name__ == "__main__":
    main()
