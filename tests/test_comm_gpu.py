"""The native communicator (csrc/comm.h) inside the training plan, one process.

RCCL refuses two ranks on one device, so on the one-GPU box the comm path runs
here as (a) a single-rank RCCL communicator (`native_comm=True`): the plan
carries the same comm-stream forks, bucket all-reduces, bf16 casts and final
join as on 8 GPUs, and a one-rank SUM all-reduce is the identity -- the step
must match an engine without communicator bit for bit (fp32) or up to the bf16
rounding of the exchanged buckets (bf16); and (b) the loopback transport, a
stand-in all-reduce that doubles each bucket in place on the comm stream: a
bucket reduced before its last (side-stream) gradient writer finished, or a
writer landing on an already-reduced range, leaves an element that is not
exactly 2x -- checked under the race check's schedule jitter too.  The world > 1
plan path (shm transport, two processes on this GPU) is in test_dp_gpu.py."""
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


def _ar_expect(persist):
    """(all-reduce ops, their streams) per plan: per-layer -- one per bucket on the comm
    stream, overlapping the backward; persistent step with persist_overlap (default) --
    the first two stage buckets on the comm stream, each behind a bucket wait, overlapping
    the backward launch, the last on the main stream after it; persistent step without --
    ONE all-reduce on the main stream after it."""
    if persist == "0":
        return None, None
    return (3, [2, 2, 0]) if "persist_overlap=0" not in persist else (1, [0])


PERSIST_MODES = ["0", "1", "1,persist_overlap=0"]


@pytest.mark.gpu
@pytest.mark.parametrize("persist", PERSIST_MODES)
def test_native_comm_single_rank_is_identity(gpu, monkeypatch, persist):
    """A one-rank SUM all-reduce is the identity: weights, momentum and gradient equal an
    engine without communicator bit for bit, for every plan shape (_ar_expect)."""
    monkeypatch.setenv("DTR_TUNE", f"persist={persist}")
    ref, eng = _engines(gpu)
    assert eng.persist == (persist != "0")
    info = eng.comm_info()
    assert info["native_rccl"], info
    n_ar, want = _ar_expect(persist)
    assert info["allreduce_ops"] >= 2 if n_ar is None else info["allreduce_ops"] == n_ar, info
    assert "librccl" in info["rccl_library"]
    names = eng.plan.names()
    assert names.count("all_reduce") == info["allreduce_ops"]
    assert names.count("prn_bucket_wait") == (2 if n_ar == 3 else 0)
    streams = eng.plan.op_streams()
    got = [streams[i] for i, n in enumerate(names) if n == "all_reduce"]
    assert got == want if want is not None else set(got) == {2}, got
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
@pytest.mark.parametrize("N,overlap", [(16, True), (48, False), (64, True), (96, False)])
def test_overlap_plan_only_where_the_reserve_costs_no_slices(gpu, monkeypatch, N, overlap):
    """The persistent overlap plan leaves 48 CUs to the comm stream; where that would cut
    the backward's slices (48 images: 4 -> 2, 96: 2 -> 1) the buckets go after the
    backward instead (train/persist.py overlap_planned)."""
    from distributed_tensorflow_resnet_amd.models.spec import build_spec
    from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule

    monkeypatch.setenv("DTR_TUNE", "persist=1")
    eng = Engine(build_spec("cifar10", 8), N, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(),
                 device=gpu, native_comm=True)
    assert eng.persist and eng.persist_overlap == overlap
    assert eng.comm_info()["allreduce_ops"] == (3 if overlap else 1)
    if eng.nat.cu_count() == 256:
        assert eng.prn.P == {16: 4, 48: 4, 64: 2, 96: 2}[N]


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


def _loopback_engines(gpu, dtype, seed_eng=3):
    import distributed_tensorflow_resnet_amd as dtr
    from distributed_tensorflow_resnet_amd.models.spec import build_spec
    from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule

    nat = dtr.native()
    spec = build_spec("cifar10", 14)
    common = dict(weight_decay=2e-4, lr_schedule=cifar_lr_schedule(), device=gpu, seed=seed_eng,
                  data_seed=11)
    ref = Engine(spec, 16, **common)
    eng = Engine(spec, 16, comm=nat.Comm.loopback(2.0), bucket_mb=0.05, allreduce_dtype=dtype,
                 **common)
    for e in (ref, eng):
        e.fill_synthetic(5)
    return ref, eng


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("persist", PERSIST_MODES)
def test_loopback_doubling_standin_orders_every_bucket(gpu, monkeypatch, dtype, persist):
    """grad == 2 x the no-comm engine's grad, bitwise, plain and under jitter (per-layer
    plan: >= 4 bucket all-reduces; persistent step: two buckets reduced and doubled on the
    comm stream WHILE the backward launch runs -- a bucket waited for too early, or a slab /
    BN gradient not yet visible when its bucket's count completed, leaves an element that
    is not exactly 2x -- and the last one after it; or all of them after it)."""
    monkeypatch.setenv("DTR_TUNE", f"persist={persist}")
    n_ar, _ = _ar_expect(persist)
    for trial in range(4):
        ref, eng = _loopback_engines(gpu, dtype)
        info = eng.comm_info()
        assert info["transport"] == "loopback", info
        assert info["allreduce_ops"] >= 4 if n_ar is None else info["allreduce_ops"] == n_ar, info
        if trial:   # schedule perturbation: random delays in front of launches, every stream
            eng.plan.set_perturb(2, 1000 + trial, 0.35, 25.0)
        ref.step()
        eng.step()
        torch.cuda.synchronize()
        base = ref.grad if dtype == "fp32" else ref.grad.to(torch.bfloat16).float()
        bad = (eng.grad != 2 * base).nonzero()
        assert bad.numel() == 0, (trial, f"{bad.numel()} elements not exactly doubled, first at "
                                  f"{bad[:4].flatten().tolist()}")


@pytest.mark.gpu
def test_racecheck_with_comm_stream_active(gpu):
    """utils/racecheck with the comm stream in the plan (bf16 exchange: casts that
    read the gradients, an all-reduce, casts back): perturbed == serialized."""
    from distributed_tensorflow_resnet_amd.utils.racecheck import _make_factory, perturbation_check

    res = perturbation_check(_make_factory("cifar_resnet14", 16, gpu, loopback=True,
                                           allreduce_dtype="bf16", bucket_mb=0.05),
                             steps=3, trials=3, prob=0.3, max_us=20.0, seed=5)
    assert res["ok"], res


@pytest.mark.gpu
def test_comm_transports_and_host_errors(gpu):
    import distributed_tensorflow_resnet_amd as dtr

    nat = dtr.native()
    assert nat.Comm.rccl_available()
    lb = nat.Comm.loopback(2.0)
    assert lb.transport == "loopback" and lb.world == 1
    x = torch.arange(1000, dtype=torch.float32, device=gpu)
    st = torch.cuda.current_stream().cuda_stream
    lb.all_reduce(x.data_ptr(), x.numel(), nat.COMM_F32, st)
    torch.cuda.synchronize()
    assert torch.equal(x, 2 * torch.arange(1000, dtype=torch.float32, device=gpu))
    # a one-rank shm communicator on the device: stream-ordered D2H / sum / H2D
    import uuid

    sh = nat.Comm.shm(f"/dtr-t-{uuid.uuid4().hex[:10]}", 1, 0, 0, slot_bytes=4096, timeout_s=10)
    y = torch.randn(5000, device=gpu)
    y0 = y.clone()
    s2 = torch.cuda.Stream()
    s2.wait_stream(torch.cuda.current_stream())
    sh.all_reduce(y.data_ptr(), y.numel(), nat.COMM_F32, s2.cuda_stream)   # 5 chunks
    sh.broadcast(y.data_ptr(), y.numel(), nat.COMM_F32, 0, s2.cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(y, y0) and sh.async_error() == 0
    sh.abort()
    assert sh.async_error() == 6
    with pytest.raises(RuntimeError):
        sh.all_reduce(y.data_ptr(), y.numel(), nat.COMM_F32, s2.cuda_stream)


@pytest.mark.gpu
def test_rccl_init_log_goes_to_its_file_and_reports_channels(gpu, tmp_path):
    """DistContext's RCCL INIT log (NCCL_DEBUG=INFO, SUBSYS=INIT, NCCL_DEBUG_FILE) must land
    in the per-process file -- never on stdout, where rank 0 prints bench.py's one JSON
    line -- and carry the channel count comm_info reports; with NCCL_MAX_NCHANNELS set
    (the persistent overlap plan's cap) RCCL builds no more channels than that."""
    log = tmp_path / "rccl.log"
    code = (
        "import torch\n"
        "from distributed_tensorflow_resnet_amd.parallel.dist import DistContext, rccl_channels_reported\n"
        "torch.cuda.set_device(0)\n"
        "comm = DistContext().native_comm(0, force=True)\n"
        "assert comm is not None\n"
        f"print('CHANNELS', rccl_channels_reported({str(log)!r}))\n")
    env = dict(os.environ, NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT", NCCL_DEBUG_FILE=str(log),
               NCCL_MAX_NCHANNELS="4")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "NCCL INFO" not in r.stdout, r.stdout[-2000:]
    assert log.exists() and "NCCL INFO" in log.read_text(), r.stdout[-2000:]
    got = [ln for ln in r.stdout.splitlines() if ln.startswith("CHANNELS")][0].split()[1]
    assert got == "None" or int(got) <= 4, got
