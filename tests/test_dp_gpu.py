"""Multi-rank data parallelism of the GPU engine, rehearsed on the one-GPU box.

RCCL refuses two ranks on one device, so these runs use DTR_DIST_BACKEND=gloo
with both ranks folded onto cuda:0, over two gradient transports:
  * c10d (default for gloo): host-issued all-reduces between plan segments;
  * shm (DTR_COMM_TRANSPORT=shm): the NATIVE world > 1 path -- bucket
    all-reduces as plan ops on the comm stream issued by its own host thread,
    event fork/join against the compute streams, bf16 casts, native
    broadcast-on-init, the init canary -- over the host-staged shared-memory
    transport that sits behind the same Comm interface as RCCL (csrc/comm_shm.cpp).
What they pin: gradients equal the exact rank-order sum of the local ones,
replicas stay identical, the bench.py multi-rank contract, and failure handling
(a killed peer makes the survivor exit non-zero fast; the launcher restarts the
job from the checkpoint).  RCCL/xGMI itself runs in the driver's 8-GPU bench."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


SHM = {"DTR_COMM_TRANSPORT": "shm"}


def _torchrun(args, port, timeout=600, extra_env=None):
    env = dict(os.environ, DTR_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.update(extra_env or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port)] + args
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.gpu
def test_dp_gradients_equal_sum_of_local_and_replicas_stay_identical(gpu):
    r = _torchrun(["scripts/dp_check.py"], 29711)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "DP_CHECK_OK" in r.stdout, r.stdout[-3000:]


@pytest.mark.gpu
def test_dp_reduce_groups_nested_in_buckets(gpu):
    # split-K reduce groups (tune reduce_mb) smaller than the all-reduce buckets:
    # several grouped reduces per bucket, the bucket joined after its last one
    r = _torchrun(["scripts/dp_check.py"], 29713,
                  extra_env={"DTR_TUNE": "reduce_mb=0.05", "DP_CHECK_BUCKET_MB": "0.5"})
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "DP_CHECK_OK" in r.stdout, r.stdout[-3000:]


@pytest.mark.gpu
def test_dp_bf16_gradient_allreduce(gpu):
    # --allreduce_dtype bf16: buckets cast into a bf16 staging buffer, all-reduced, cast back
    r = _torchrun(["scripts/dp_check.py"], 29714, extra_env={"DP_CHECK_ALLREDUCE": "bf16"})
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "DP_CHECK_OK" in r.stdout, r.stdout[-3000:]


@pytest.mark.gpu
def test_bench_two_ranks_contract(gpu):
    r = _torchrun(["bench.py", "--gpus", "2", "--steps", "5", "--warmup", "2"], 29712)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 5 and out["config"]["global_batch"] == 128
    assert out["config"]["per_gpu_batch"] == 64 and out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,port", [("fp32", 29721), ("bf16", 29722)])
def test_native_plan_path_two_ranks_shm(gpu, dtype, port):
    r = _torchrun(["scripts/dp_check.py"], port,
                  extra_env=dict(SHM, DP_CHECK_ALLREDUCE=dtype, DP_CHECK_BUCKET_MB="0.1"))
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "DP_CHECK_OK" in r.stdout, r.stdout[-3000:]
    assert "transport=shm native=True" in r.stdout and "fallback=None" in r.stdout, r.stdout[-2000:]


@pytest.mark.gpu
def test_bench_self_spawn_two_ranks_native_shm(gpu):
    """`bench.py --gpus 2` (self-spawned ranks) over the native plan path."""
    env = dict(os.environ, DTR_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", **SHM)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "6", "--warmup", "3",
                        "--model", "cifar_resnet20"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    c = out["config"]["comm"]
    assert c["native"] and c["transport"] == "shm" and c["fallback_reason"] is None, c
    assert c["allreduce_ops"] >= 2 and c["buckets"] == c["allreduce_ops"], c
    assert out["n_gpus"] == 2 and out["pg_world_size"] == 2
    assert out["phase_ms"]["allreduce_exposed"] >= 0.0


def _spawn_ranks(args, port, extra_env):
    procs = []
    for rank in range(2):
        env = dict(os.environ, DTR_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0",
                   RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE="2", LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **extra_env)
        procs.append(subprocess.Popen([sys.executable] + args, cwd=ROOT, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    return procs


@pytest.mark.gpu
def test_killed_peer_makes_survivor_exit_nonzero_fast(gpu, tmp_path):
    """Rank 1 dies at step 3 (fault injection); rank 0, with no launcher to stop
    it, must notice inside its next gradient all-reduce and exit non-zero well
    before the 120 s collective timeout."""
    import time

    args = ["resnet_cifar_main.py", "--device", "gpu", "--resnet_size", "8", "--batch_size", "8",
            "--synthetic", "--train_steps", "50", "--variable_update", "horovod",
            "--log_every", "1000", "--comm_timeout_secs", "120", "--fault_kill_step", "3",
            "--fault_kill_rank", "1"]
    t0 = time.time()
    procs = _spawn_ranks(args, 29731, SHM)
    try:
        out1, _ = procs[1].communicate(timeout=240)
        t1 = time.time()
        out0, _ = procs[0].communicate(timeout=200)
        t_exit = time.time() - t1
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert procs[1].returncode == 17, out1[-2000:]
    assert procs[0].returncode != 0, out0[-3000:]
    assert t_exit < 60, f"survivor exited {t_exit:.0f}s after the peer died"
    assert "is gone" in out0 or "aborted by rank" in out0, out0[-3000:]
    assert time.time() - t0 < 400


@pytest.mark.gpu
def test_launcher_restarts_native_job_from_checkpoint(gpu, tmp_path):
    """2 ranks on the native shm path: rank 1 killed at step 3, the launcher
    restarts the job, the ranks resume from the step-2 checkpoint and finish."""
    import distributed_tensorflow_resnet_amd.utils.tensor_bundle as tb

    td = str(tmp_path / "train")
    env = dict(os.environ, DTR_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", **SHM)
    r = subprocess.run([sys.executable, "-m", "distributed_tensorflow_resnet_amd.parallel.launch",
                        "--nproc", "2", "--master_port", "29741", "--max_restarts", "1",
                        "resnet_cifar_main.py", "--device", "gpu", "--resnet_size", "8",
                        "--batch_size", "8", "--synthetic", "--train_steps", "6",
                        "--train_dir", td, "--save_checkpoint_steps", "2",
                        "--variable_update", "horovod", "--log_every", "1",
                        "--comm_timeout_secs", "120",
                        "--fault_kill_step", "3", "--fault_kill_rank", "1"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "restarting job" in r.stdout and "Restoring parameters from" in r.stdout, r.stdout[-3000:]
    assert tb.latest_checkpoint(td).endswith("model.ckpt-6")


# Two ranks on ONE GPU with disjoint halves of its CUs (DTR_CU_PARTITION=2 ->
# ROC_GLOBAL_CU_MASK per process): each rank may then run the persistent step's
# co-resident grids, sized by its masked CU count (128), so the world > 1 headline path
# -- the persistent backward with the overlap plan's 48-CU reserve, the comm stream's
# bucket waits, packs, all-reduces and early parameter updates beside it -- runs with a
# real second rank and a real cross-process exchange (the shm transport: RCCL refuses
# two ranks on one device).  bs16 per rank = the 8-GPU share of the global batch 128.
CUP = dict(SHM, DTR_CU_PARTITION="2")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,port", [("fp32", 29751), ("bf16", 29752)])
def test_persistent_overlap_two_ranks_cu_partition(gpu, dtype, port):
    r = _torchrun(["scripts/dp_check.py"], port, timeout=600,
                  extra_env=dict(CUP, DP_CHECK_SIZE="50", DP_CHECK_BATCH="16",
                                 DP_CHECK_STEPS="20", DP_CHECK_ALLREDUCE=dtype))
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "DP_CHECK_OK" in r.stdout, r.stdout[-3000:]
    assert "step_path=persistent(P=4/4,overlap=1" in r.stdout, r.stdout[-2000:]
    assert "transport=shm native=True" in r.stdout and "cus=128" in r.stdout, r.stdout[-2000:]
    assert "persist_errors=0" in r.stdout, r.stdout[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,port", [("fp32", 29753), ("bf16", 29754)])
def test_imagenet_plan_two_ranks_cu_partition(gpu, dtype, port):
    """The ImageNet per-layer plan at world 2 (ResNet-50, 16 images per rank, CU halves,
    shm transport): main + side streams and four 25 MB comm-stream buckets; the all-reduced
    gradient is the exact rank-order sum and the replicas stay identical."""
    r = _torchrun(["scripts/dp_check.py"], port, timeout=600,
                  extra_env=dict(CUP, DP_CHECK_DATASET="imagenet", DP_CHECK_SIZE="50",
                                 DP_CHECK_BATCH="16", DP_CHECK_BUCKET_MB="25",
                                 DP_CHECK_STEPS="10", DP_CHECK_ALLREDUCE=dtype))
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "DP_CHECK_OK" in r.stdout, r.stdout[-3000:]
    assert "allreduce_ops=4" in r.stdout and "step_path=per-layer" in r.stdout, r.stdout[-2000:]


@pytest.mark.gpu
def test_bench_two_ranks_persistent_cu_partition(gpu):
    """`bench.py --gpus 2` on the persistent step at world 2 (CU halves, shm transport)."""
    env = dict(os.environ, DTR_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", **CUP)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "20", "--warmup", "5",
                        "--batch", "32"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=400)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    cfg = out["config"]
    assert out["pg_world_size"] == 2 and cfg["per_gpu_batch"] == 16, out
    assert cfg["step_path"].startswith("persistent") and cfg["persist_overlap"], cfg
    assert cfg["cus"] == 128 and cfg["comm"]["transport"] == "shm", cfg


@pytest.mark.gpu
def test_bench_four_ranks_persistent_cu_quarters(gpu):
    """`bench.py --gpus 4` with four ranks on CU quarters (64 CUs each, 32 images per rank):
    the overlap plan's 48-CU reserve does not fit beside the grid, so each rank takes the
    persistent step with the buckets after the backward (train/persist.py overlap_planned)
    rather than the per-layer plan."""
    env = dict(os.environ, DTR_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0",
               **dict(SHM, DTR_CU_PARTITION="4"))
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--steps", "20", "--warmup", "5"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    cfg = out["config"]
    assert out["pg_world_size"] == 4 and cfg["per_gpu_batch"] == 32 and cfg["cus"] == 64, out
    assert cfg["step_path"].startswith("persistent") and not cfg["persist_overlap"], cfg


@pytest.mark.gpu
def test_bench_two_ranks_falls_back_after_a_persistent_fault(gpu):
    """bench.py at world > 1: a persistent-step barrier timeout on ONE rank (rank 1's lost
    workgroup, DTR_PRN_FAULT_BAR=3@1) is agreed over the process group and the job
    measures again on the next plan down -- persistent without the overlap (which faults
    again: the injection stays on), then the per-layer plan -- and reports that number
    with the fallback chain instead of no number."""
    env = dict(os.environ, DTR_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0",
               DTR_TEST_FAULTS="1", DTR_PRN_FAULT_BAR="3@1", **CUP)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "10", "--warmup", "3",
                        "--batch", "32"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=400)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    cfg = out["config"]
    assert cfg["step_path"] == "per-layer plan", cfg
    assert cfg["fallback"] and len(cfg["fallback"]) == 2, cfg
    assert "persist_overlap=0" in cfg["fallback"][1], cfg
    assert out["value"] > 0 and out["pg_world_size"] == 2, out


@pytest.mark.gpu
def test_fault_on_one_rank_fails_job_and_restarts_per_layer(gpu, tmp_path):
    """a grid-barrier timeout on a NON-chief rank (DTR_PRN_FAULT_BAR=3@1) must
    fail the whole job before the chief checkpoints the poisoned state: the faulting rank
    raises at its next health read and writes the marker; the restart resumes from the
    last agreed checkpoint on the per-layer plan and finishes."""
    import distributed_tensorflow_resnet_amd.utils.tensor_bundle as tb

    td = str(tmp_path / "train")
    common = ["resnet_cifar_main.py", "--device", "gpu", "--resnet_size", "8", "--batch_size", "16",
              "--synthetic", "--train_dir", td, "--save_checkpoint_steps", "1",
              "--variable_update", "horovod", "--log_every", "1", "--comm_timeout_secs", "120"]
    env = dict(os.environ, DTR_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0", **CUP)
    launch = [sys.executable, "-m", "distributed_tensorflow_resnet_amd.parallel.launch", "--nproc", "2"]
    r = subprocess.run(launch + ["--master_port", "29761"] + common + ["--train_steps", "2"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert tb.latest_checkpoint(td).endswith("model.ckpt-2")
    env.update(DTR_PRN_FAULT_BAR="3@1", DTR_TEST_FAULTS="1")
    r = subprocess.run(launch + ["--master_port", "29771", "--max_restarts", "1"] + common +
                       ["--train_steps", "4"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=500)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "grid barrier timed out" in out and "[launch] a rank failed" in out, out[-4000:]
    assert "persistent step disabled" in out, out[-4000:]
    assert os.path.exists(os.path.join(td, "persist_fault"))
    # written by the faulting rank 1 and by rank 0 once the agreement failed (last wins)
    marker = open(os.path.join(td, "persist_fault")).read()
    assert "rank 1 at step 3" in marker or "rank 0 at step 3" in marker and "another rank" in marker
    # the broken step never reached a checkpoint: both attempts resumed from step 2
    assert out.count("(global_step=2)") == 4, out[-4000:]   # 2 ranks x 2 attempts
    assert tb.latest_checkpoint(td).endswith("model.ckpt-4")
