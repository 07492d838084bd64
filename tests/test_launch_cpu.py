"""The launch/ shell scripts (MI355X equivalents of the reference's docker /
mpirun / SLURM launchers) on the CPU: syntax of every script, the localhost gloo
pseudo-cluster, and start -> checkpoint -> stop of a background run with its
side-car evaluator."""
import glob
import os
import subprocess
import time

import pytest

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

    assert [slices_for(n, 256) for n in (8, 16, 32, 48, 56, 64, 96, 112, 128, 224)] == [4, 4, 4, 4, 4, 2, 2, 1, 1, 1]
    assert [slices_for(n, 128) for n in (16, 24, 32, 48, 96)] == [4, 4, 2, 2, 1]
    # a rank on a CU half after the overlap reserve (128 - 48)
    assert [slices_for(n, 80) for n in (8, 16, 24, 32, 64)] == [4, 4, 2, 2, 1]
    assert [fwd_slices_for(n, 256) for n in (8, 16, 32, 40, 47, 48, 64, 96, 120, 128, 200)] == [4, 4, 4, 4, 4, 2, 2, 2, 2, 1, 1]
    assert slices_for(128, 256, 2) == 2 and fwd_slices_for(16, 256, 1) == 1
    for n in range(1, 241):
        assert n * slices_for(n, 256) + 16 <= 256
        assert n * fwd_slices_for(n, 256) <= 256


def test_cu_partition_masks_and_disjoint_sharing(monkeypatch):
    """DTR_CU_PARTITION: disjoint contiguous CU masks per rank (ROC_GLOBAL_CU_MASK), and
    ranks on one GPU whose masks are disjoint do not count as sharing it (VERDICT r5
    item 1: the two-rank rehearsal of the persistent step), overlapping masks do."""
    import torch
    import torch.distributed as dist

    from distributed_tensorflow_resnet_amd.parallel import dist as D

    assert D.cu_partition_mask(0, 2, 256) == (1 << 128) - 1
    assert D.cu_partition_mask(1, 2, 256) == ((1 << 128) - 1) << 128
    assert D.cu_partition_mask(3, 4, 256) >> 192 == (1 << 64) - 1
    with pytest.raises(ValueError):
        D.cu_partition_mask(2, 2, 256)
    monkeypatch.delenv("ROC_GLOBAL_CU_MASK", raising=False)
    monkeypatch.setenv("DTR_CU_PARTITION", "")
    assert D.apply_cu_partition() is None and "ROC_GLOBAL_CU_MASK" not in os.environ
    monkeypatch.setattr(D, "_kfd_cu_count", lambda: 256)
    monkeypatch.setenv("DTR_CU_PARTITION", "2")
    monkeypatch.setenv("LOCAL_RANK", "1")
    assert D.apply_cu_partition() == hex(((1 << 128) - 1) << 128) == os.environ["ROC_GLOBAL_CU_MASK"]
    monkeypatch.setenv("DTR_CU_PARTITION", "0/4")
    assert int(D.apply_cu_partition(), 16) == (1 << 64) - 1

    # sharing over a store: rank 0 and 1 on GPU "x"; disjoint masks -> not shared
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)
    monkeypatch.setattr(D, "device_identity", lambda i: "x")
    store = dist.HashStore()
    monkeypatch.setattr(dist.distributed_c10d, "_get_default_store", lambda: store, raising=False)
    ctx = type("C", (), {"active": True, "rank": 0, "world_size": 2})()
    store.set("dtr/dev/1", f"{D.socket.gethostname()}|x")
    store.set("dtr/cumask/1", "%x" % (((1 << 128) - 1) << 128))
    monkeypatch.setattr(D, "_cu_mask_int", lambda: (1 << 128) - 1)
    assert not D.gpu_shared_by_ranks(ctx, 0)
    monkeypatch.setattr(D, "_cu_mask_int", lambda: (1 << 256) - 1)   # no partition: every CU
    assert D.gpu_shared_by_ranks(ctx, 0)
    store.set("dtr/dev/1", f"{D.socket.gethostname()}|y")   # the peer on another GPU
    assert not D.gpu_shared_by_ranks(ctx, 0)


def test_persist_fault_marker_lifecycle(tmp_path, monkeypatch):
    """the persist_fault marker turns the persistent step off (DTR_TUNE
    persist=0, the reason returned for metrics.jsonl), --reset_persist_fault deletes it so
    the persistent step may be selected again."""
    from distributed_tensorflow_resnet_amd.train import driver
    from distributed_tensorflow_resnet_amd.utils.flags import build_parser

    td = tmp_path / "train"
    td.mkdir()
    (td / driver.PERSIST_FAULT_MARKER).write_text("rank 1 at step 3: barrier timed out\n")
    monkeypatch.setenv("DTR_TUNE", "")
    flags = build_parser("cifar").parse_args(["--train_dir", str(td)])
    why = driver.persist_fault_policy(flags)
    assert "rank 1 at step 3" in why and "persist=0" in os.environ["DTR_TUNE"]
    monkeypatch.setenv("DTR_TUNE", "")
    flags = build_parser("cifar").parse_args(["--train_dir", str(td), "--reset_persist_fault"])
    assert driver.persist_fault_policy(flags) == ""
    assert not (td / driver.PERSIST_FAULT_MARKER).exists() and os.environ["DTR_TUNE"] == ""


def test_persist_health_hook_agrees_and_gates_saves():
    """the health agreement raises on EVERY rank when any rank's persistent
    launch failed, and the checkpoint hook saves only agreed steps."""
    from distributed_tensorflow_resnet_amd.train import hooks as H
    from distributed_tensorflow_resnet_amd.train.engine import PersistentStepError

    class Ctx:
        def __init__(self, others_ok):
            self.others_ok = others_ok

        def _agree(self, ok):
            return ok and self.others_ok

    class Eng:
        err = False

        def persist_error(self):
            return self.err

    class Saver:
        saved = []

        def save(self, t, step):
            self.saved.append(step)
            return f"ckpt-{step}"

    sess = type("S", (), {})()
    sess.backend = type("B", (), {"engine": Eng()})()
    sess.is_chief = True
    sess.state_tensors = lambda: {}
    sess.global_step = 0
    hh = H.PersistHealthHook(Ctx(True), every=2)
    ck = H.CheckpointSaverHook(Saver(), save_steps=0, save_secs=1e-9)
    hh.begin(sess)
    ck.begin(sess)
    for step in (1, 2, 3):
        hh.after_run(sess, step)
        ck.after_run(sess, step)
    assert Saver.saved == [2]            # the time-based save waited for the agreed step 2
    hh = H.PersistHealthHook(Ctx(False), every=1)   # another rank's flag is set
    with pytest.raises(PersistentStepError, match="another rank"):
        hh.after_run(sess, 4)


def test_rccl_channel_log_parse(tmp_path):
    """comm_info's rccl_channels: the largest `Channel xx/NN` of RCCL's INIT log."""
    from distributed_tensorflow_resnet_amd.parallel.dist import rccl_channels_reported

    p = tmp_path / "rccl.log"
    p.write_text("host:1:1 [0] NCCL INFO Channel 00/32 :    0   1   2   3   4   5   6   7\n"
                 "host:1:1 [0] NCCL INFO Channel 31/32 :    0   1   2   3   4   5   6   7\n"
                 "host:1:1 [0] NCCL INFO Channel 00/24 :    0   1\n")
    assert rccl_channels_reported(str(p)) == 32
    assert rccl_channels_reported(str(tmp_path / "missing")) is None
    assert rccl_channels_reported(None) is None
