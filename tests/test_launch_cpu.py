"""The launch/ shell scripts (MI355X equivalents of the reference's docker /
mpirun / SLURM launchers) on the CPU: syntax of every script, the localhost gloo
pseudo-cluster, and start -> checkpoint -> stop of a background run with its
side-car evaluator."""
import glob
import os
import subprocess
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_scripts_parse():
    files = glob.glob(os.path.join(ROOT, "launch", "*.sh")) + \
        glob.glob(os.path.join(ROOT, "launch", "slurm", "*.sbatch"))
    assert len(files) >= 9
    for f in files:
        r = subprocess.run(["bash", "-n", f], capture_output=True, text=True)
        assert r.returncode == 0, (f, r.stderr)


def test_local_cpu_pseudo_cluster(tmp_path):
    env = dict(os.environ, NPROC="2", STEPS="3", RUN_DIR=str(tmp_path), MASTER_PORT="29643",
               LOG_EVERY="1", SAVE_STEPS="3")
    r = subprocess.run(["bash", os.path.join(ROOT, "launch", "run_local_cpu.sh")], env=env,
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    assert os.path.exists(tmp_path / "ckpt" / "checkpoint")


def test_start_and_stop_background_run(tmp_path):
    env = dict(os.environ, GPUS="2", GLOBAL_BATCH="8", RESNET_SIZE="8", TRAIN_STEPS="1000000",
               DEVICE="cpu", RUN_DIR=str(tmp_path), MASTER_PORT="29644", SYNTHETIC="1",
               EXTRA_ARGS="--dtype fp32 --save_checkpoint_steps 2 --log_every 1")
    r = subprocess.run(["bash", os.path.join(ROOT, "launch", "start-resnet-cifar-main.sh")],
                       env=env, capture_output=True, text=True, timeout=60, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    pids = {os.path.basename(f)[:-4]: int(open(f).read()) for f in
            glob.glob(str(tmp_path / "*.pid"))}
    assert set(pids) == {"train", "eval"}
    try:
        deadline = time.time() + 300
        while time.time() < deadline and not os.path.exists(tmp_path / "ckpt" / "checkpoint"):
            time.sleep(1)
        assert os.path.exists(tmp_path / "ckpt" / "checkpoint"), \
            open(tmp_path / "logs" / "train.log").read()[-3000:]
    finally:
        s = subprocess.run(["bash", os.path.join(ROOT, "launch", "stop.sh"), str(tmp_path)],
                           capture_output=True, text=True, timeout=120)
    assert s.returncode == 0, s.stderr
    for pid in pids.values():
        try:
            os.kill(pid, 0)
            alive = True
        except ProcessLookupError:
            alive = False
        assert not alive
    assert not glob.glob(str(tmp_path / "*.pid"))


def test_gpu_shared_by_ranks(monkeypatch):
    """Ranks folded onto fewer GPUs than ranks (one-GPU rehearsals) must switch the
    persistent CIFAR step off: its grids need every CU of the device to themselves."""
    import torch

    from distributed_tensorflow_resnet_amd.parallel.dist import gpu_shared_by_ranks

    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    assert gpu_shared_by_ranks()
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    assert not gpu_shared_by_ranks()
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    assert not gpu_shared_by_ranks()
    monkeypatch.delenv("LOCAL_WORLD_SIZE")
    monkeypatch.setenv("WORLD_SIZE", "16")
    assert gpu_shared_by_ranks()
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 0)
    assert not gpu_shared_by_ranks()


def test_persistent_slice_selection():
    """Row slices per image of the persistent CIFAR step (train/persist.py): the backward
    leaves >= 32 CUs for the weight-gradient workgroups, the forward may fill the chip,
    and tune persist_slices overrides both."""
    from distributed_tensorflow_resnet_amd.train.persist import fwd_slices_for, slices_for

    assert [slices_for(n, 256) for n in (8, 16, 32, 48, 64, 96, 128, 224)] == [4, 4, 4, 2, 2, 1, 1, 1]
    assert [fwd_slices_for(n, 256) for n in (8, 16, 32, 48, 64, 96, 128, 200)] == [4, 4, 4, 2, 2, 2, 1, 1]
    assert slices_for(128, 256, 2) == 2 and fwd_slices_for(16, 256, 1) == 1
    for n in range(1, 241):
        assert n * slices_for(n, 256) + 16 <= 256
        assert n * fwd_slices_for(n, 256) <= 256
