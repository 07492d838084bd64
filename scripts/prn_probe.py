"""Phase timeline of the persistent CIFAR launches (csrc/cifar_persist.hip): image 0's
lane 0 stamps the wall clock (100 MHz) at every phase boundary; this prints, per
phase transition, the mean and total time over all blocks of the forward and of the
backward launch.  python scripts/prn_probe.py [batch] [resnet_size]"""
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("DTR_TUNE", "persist=1")
from distributed_tensorflow_resnet_amd.models.spec import cifar_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule  # noqa: E402

NAMES = {
    "fwd": {0: "start", 99: "prev block: tail", 1: "BN1 table+halo", 2: "BN1 sync", 3: "conv1", 4: "publish+stats", 5: "arrive",
            6: "wait", 8: "BN2 combine+halo+wstore+sync", 9: "conv2", 10: "publish+stats",
            11: "arrive", 12: "wait+wstore", 200: "blocks done"},
    "bwd": {0: "start", 1: "loads+publish+sync", 3: "conv2 dgrad", 99: "prev block: wstore+tail", 4: "publish+bwd sums", 5: "arrive", 6: "wait",
            8: "BN2 combine+apply+halo+wstore+sync", 9: "conv1 dgrad", 10: "publish+bwd sums",
            11: "arrive", 12: "wait", 13: "BN1 table (sums read)", 14: "BN1 apply",
            15: "BN1 halo", 200: "blocks done"},
}


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    eng = Engine(cifar_spec(size), N, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(),
                 device=torch.device("cuda", 0))
    assert eng.persist
    wgs = os.environ.get("PRN_WGRAD_WGS")   # diagnostics: rebuild the plan with fewer
    if wgs:                                 # weight-gradient workgroups
        eng.prn.wgrad_wgs = int(wgs)
        eng.plan = eng.nat.Plan()
        eng._keep = []
        eng._build_train_plan()
    print(f"slices per image {eng.prn.P}, weight-gradient workgroups {eng.prn.wgrad_wgs}, "
          f"items {len(eng.prn.items)}")
    eng.fill_synthetic(0)
    for _ in range(20):
        eng.step()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream().cuda_stream
    for seg in ("fwd", "bwd"):
        buf = torch.zeros(2 * 4096, dtype=torch.int64, device="cuda")
        eng.nat.prn_set_probe(buf.data_ptr())
        for _ in range(3):   # the last run's stamps
            buf.zero_()
            eng.nat.prn_set_probe(0)
            eng._run("fwd", st)
            if seg == "bwd":
                eng.nat.prn_set_probe(buf.data_ptr())
            eng._run_bwd(st)
            torch.cuda.synchronize()
        eng.nat.prn_set_probe(0)
        if seg == "fwd":   # re-run the forward alone with the probe on
            buf.zero_()
            eng.nat.prn_set_probe(buf.data_ptr())
            eng._run("fwd", st)
            torch.cuda.synchronize()
            eng.nat.prn_set_probe(0)
        last_item = int(buf[8191].item())
        buf[8191] = 0
        v = buf.view(-1, 2).cpu().tolist()
        stamps = [(t, c) for t, c in v if c != 0]
        if seg == "bwd" and last_item:
            print(f"  (weight-gradient workgroups out of items {(last_item - stamps[-1][1]) / 100.0:+.1f} us "
                  f"after slice 0's last stamp)")
        acc = defaultdict(list)
        for (t0, c0), (t1, c1) in zip(stamps, stamps[1:]):
            if t1 >= 100 and t1 < 200:
                t1 = 99
            acc[t1].append((c1 - c0) / 100.0)
        total = (stamps[-1][1] - stamps[0][1]) / 100.0
        print(f"== {seg} (N={N}, resnet{size}): {total:.1f} us from first to last stamp")
        for t in sorted(acc):
            xs = acc[t]
            print(f"  {str(NAMES[seg].get(t, t)):34s} n={len(xs):3d} mean {sum(xs)/len(xs):7.2f} us  total {sum(xs):8.1f} us")
        stage_t = defaultdict(float)
        per = defaultdict(lambda: defaultdict(list))   # phase -> stage -> [us]
        cur = None
        for (t0, c0), (t1, c1) in zip(stamps, stamps[1:]):
            if t0 >= 100 and t0 < 200:
                cur = t0 - 100
            if cur is not None:
                stage_t[cur] += (c1 - c0) / 100.0
                if not (100 <= t1 < 200):
                    per[t1][cur].append((c1 - c0) / 100.0)
        print("  per stage:", {k: round(v, 1) for k, v in sorted(stage_t.items())})
        print("  mean us per phase and stage:")
        for t in sorted(per):
            row = "  ".join(f"s{k}: {sum(v) / len(v):5.2f}" for k, v in sorted(per[t].items()))
            print(f"    {str(NAMES[seg].get(t, t)):34s} {row}")
    step = eng.step_timed()
    print("step_timed:", {k: round(v, 4) for k, v in step.items()})


if __name__ == "__main__":
    main()
