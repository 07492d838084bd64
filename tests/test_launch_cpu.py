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
    """Ranks on one physical GPU (one-GPU rehearsals) must switch the persistent CIFAR
    step off -- its grids need every CU of the device to themselves -- and ranks that
    each see one GPU through a visible-device mask (ordinal 0 everywhere) must not be
    mistaken for sharing: the decision comes from physical device identities
    exchanged through the c10d store."""
    import types

    import torch
    import torch.distributed as dist

    from distributed_tensorflow_resnet_amd.parallel import dist as D

    # identities: PCI location first, then the UUID, then the visible masks + ordinal
    props = types.SimpleNamespace(pci_domain_id=0, pci_bus_id=0x15, pci_device_id=0, uuid="abc")
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda i: props)
    assert D.device_identity(0) == "pci:0:15:0"
    props = types.SimpleNamespace(uuid="GPU-1234")
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda i: props)
    assert D.device_identity(0) == "uuid:GPU-1234"
    props = types.SimpleNamespace(uuid="00000000-0000-0000-0000-000000000000")
    monkeypatch.setattr(torch.cuda, "get_device_properties", lambda i: props)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "3")
    a = D.device_identity(0)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "5")
    assert D.device_identity(0) != a          # one GPU per rank by mask: distinct

    # counting over a store: ranks 0 and 1 share GPU "x", rank 2 has "y"
    store = dist.HashStore()
    store.set("dtr/t/1", f"{D.socket.gethostname()}|x")
    store.set("dtr/t/2", f"{D.socket.gethostname()}|y")
    assert D.ranks_on_device(store, 0, 3, "x", tag="t") == 2
    store = dist.HashStore()
    store.set("dtr/u/0", f"{D.socket.gethostname()}|x")
    store.set("dtr/u/1", "otherhost|y")
    assert D.ranks_on_device(store, 2, 3, "y", tag="u") == 1   # same id on another host
    # no process group: never shared
    assert not D.gpu_shared_by_ranks(None)


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
