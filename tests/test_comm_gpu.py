"""The native RCCL communicator (csrc/comm.h) inside the training plan.

RCCL refuses two ranks on one device, so on the one-GPU box the comm path runs
as a single-rank communicator (`native_comm=True`): the plan carries the same
comm-stream forks, bucket all-reduces, bf16 casts and final join as on 8 GPUs,
and a one-rank SUM all-reduce is the identity -- so the step must match an
engine without communicator bit for bit (fp32) or up to the bf16 rounding of
the exchanged buckets (bf16).  Multi-rank RCCL runs in the driver's 8-GPU
scaling bench; the multi-rank logic is rehearsed over gloo in test_dp_gpu.py."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _engines(gpu, **kw):
    from distributed_tensorflow_resnet_amd.models.spec import build_spec
    from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule

    spec = build_spec("cifar10", 14)
    common = dict(weight_decay=2e-4, lr_schedule=cifar_lr_schedule(), device=gpu, seed=3,
                  data_seed=11)
    ref = Engine(spec, 16, **common)
    eng = Engine(spec, 16, native_comm=True, bucket_mb=0.05, **common, **kw)
    for e in (ref, eng):
        e.fill_synthetic(5)
    return ref, eng


@pytest.mark.gpu
def test_native_comm_single_rank_is_identity(gpu):
    ref, eng = _engines(gpu)
    info = eng.comm_info()
    assert info["native_rccl"] and info["allreduce_ops"] >= 2, info
    assert "librccl" in info["rccl_library"]
    names = eng.plan.names()
    assert names.count("all_reduce") == info["allreduce_ops"]
    streams = eng.plan.op_streams()
    assert all(streams[i] == 2 for i, n in enumerate(names) if n == "all_reduce")
    for _ in range(3):
        ref.step()
        eng.step()
    torch.cuda.synchronize()
    assert torch.equal(ref.grad, eng.grad)
    assert torch.equal(ref.params.master, eng.params.master)
    assert torch.equal(ref.mom, eng.mom)
    ph = eng.step_timed()
    assert ph["allreduce_exposed"] >= 0.0 and ph["backward"] > 0.0


@pytest.mark.gpu
def test_native_comm_bf16_exchange(gpu):
    ref, eng = _engines(gpu, allreduce_dtype="bf16")
    assert eng.comm_info()["allreduce_bytes"] == 2 * eng.params.n_train
    ref.step()
    eng.step()
    torch.cuda.synchronize()
    want = ref.grad.to(torch.bfloat16).float()   # one rank: exactly the bf16 rounding
    assert torch.equal(want, eng.grad)


@pytest.mark.gpu
def test_native_comm_broadcast_and_errors(gpu):
    import distributed_tensorflow_resnet_amd as dtr

    nat = dtr.native()
    comm = nat.Comm(nat.Comm.unique_id(), 1, 0, 0)
    x = torch.arange(1000, dtype=torch.float32, device=gpu)
    st = torch.cuda.current_stream().cuda_stream
    comm.broadcast(x.data_ptr(), x.numel(), nat.COMM_F32, 0, st)
    comm.all_reduce(x.data_ptr(), x.numel(), nat.COMM_F32, st)
    torch.cuda.synchronize()
    assert torch.equal(x, torch.arange(1000, dtype=torch.float32, device=gpu))
    assert comm.async_error() == 0
    with pytest.raises(ValueError):
        nat.Comm(b"short", 1, 0, 0)
    comm.abort()
    with pytest.raises(RuntimeError):
        comm.all_reduce(x.data_ptr(), x.numel(), nat.COMM_F32, st)


@pytest.mark.gpu
def test_bench_self_spawn_two_gloo_ranks(gpu):
    """`python bench.py --gpus 2` outside torchrun spawns its own rank processes
    (both folded onto this GPU over gloo) and reports the process group's size."""
    env = dict(os.environ, DTR_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "4", "--warmup", "2",
                        "--model", "cifar_resnet20"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["pg_world_size"] == 2 and out["dist_backend"] == "gloo"
    assert out["config"]["per_gpu_batch"] == 64 and out["config"]["comm"]["buckets"] >= 1
    assert out["phase_ms"]["allreduce_exposed"] >= 0.0
