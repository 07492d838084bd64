"""The training driver on the GPU engine: train (hipGraph) -> TF checkpoint ->
resume on the GPU -> side-car eval on the GPU -> resume the same checkpoint on
the CPU backend (cross-backend checkpoint compatibility)."""
import glob
import os
import subprocess
import sys

import pytest

from distributed_tensorflow_resnet_amd.utils import records
from distributed_tensorflow_resnet_amd.utils import tensor_bundle as tb

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(args, env=None, timeout=600):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([sys.executable] + args, cwd=ROOT, capture_output=True, text=True,
                          timeout=timeout, env=e)


def test_driver_gpu_train_resume_eval(gpu, tmp_path):
    td, ld, ed = (str(tmp_path / d) for d in ("train", "log", "eval"))
    common = ["--device", "gpu", "--synthetic", "--resnet_size", "20", "--batch_size", "64",
              "--train_dir", td, "--log_dir", ld, "--log_every", "10", "--summary_every", "10",
              "--save_checkpoint_steps", "25"]
    r = run(["resnet_cifar_main.py", "--train_steps", "50"] + common)
    assert r.returncode == 0, r.stderr[-4000:]
    assert tb.latest_checkpoint(td).endswith("model.ckpt-50")
    assert "step = 50" in r.stdout
    evs = records.read_events(glob.glob(os.path.join(ld, "events.out.tfevents.*"))[0])
    costs = [e["scalars"]["cost"] for e in evs if "cost" in e["scalars"]]
    assert len(costs) >= 4 and costs[-1] < costs[0]
    r = run(["resnet_cifar_main.py", "--train_steps", "60", "--profile_steps", "52:56"] + common)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "Restoring parameters from" in r.stdout and "phase timing" in r.stdout
    assert tb.latest_checkpoint(td).endswith("model.ckpt-60")
    r = run(["resnet_cifar_eval.py", "--device", "gpu", "--synthetic", "--resnet_size", "20",
             "--train_dir", td, "--eval_dir", ed, "--eval_once", "--eval_batch_count", "3"])
    assert r.returncode == 0, r.stderr[-4000:]
    assert "best precision" in r.stdout
    r = run(["resnet_cifar_main.py", "--device", "cpu", "--synthetic", "--resnet_size", "20",
             "--batch_size", "8", "--train_dir", td, "--train_steps", "61"],
            env={"HIP_VISIBLE_DEVICES": ""})
    assert r.returncode == 0, r.stderr[-4000:]
    assert "Restoring parameters from" in r.stdout
    assert tb.latest_checkpoint(td).endswith("model.ckpt-61")


def test_imagenet_driver_gpu_synthetic(gpu, tmp_path):
    r = run(["resnet_imagenet_main.py", "--device", "gpu", "--synthetic", "--resnet_size", "50",
             "--batch_size", "32", "--train_steps", "6", "--log_every", "3"])
    assert r.returncode == 0, r.stderr[-4000:]
    assert "training precision" in r.stdout


def test_persistent_fault_fails_job_and_restart_falls_back(gpu, tmp_path):
    """A persistent CIFAR launch whose grid barrier times out must fail the job, not the
    model: DTR_PRN_FAULT_BAR makes forward workgroup 0 abandon the
    launch at its 3rd barrier (a lost workgroup; the others time out at the next one).
    The first metrics read raises, the CLI exits 3 WITHOUT writing a checkpoint of the
    broken step and leaves the fault marker; the launcher's restart resumes from the
    last good checkpoint on the per-layer plan and finishes."""
    td = str(tmp_path / "train")
    common = ["--device", "gpu", "--synthetic", "--resnet_size", "8", "--batch_size", "16",
              "--train_dir", td, "--log_every", "1", "--save_checkpoint_steps", "1"]
    r = run(["resnet_cifar_main.py", "--train_steps", "2"] + common)
    assert r.returncode == 0, r.stderr[-4000:]
    assert tb.latest_checkpoint(td).endswith("model.ckpt-2")
    r = run(["-m", "distributed_tensorflow_resnet_amd.parallel.launch", "--nproc", "1",
             "--max_restarts", "1", "--master_port", "29634", "resnet_cifar_main.py",
             "--train_steps", "4"] + common, env={"DTR_PRN_FAULT_BAR": "3", "DTR_TEST_FAULTS": "1"})
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "grid barrier timed out" in out and "exiting with code 3" in out, out[-4000:]
    assert "[launch] a rank failed with exit code 3" in out
    assert "persistent step disabled" in out
    assert os.path.exists(os.path.join(td, "persist_fault"))
    # the broken step 3 never reached a checkpoint: both attempts resumed from step 2
    assert out.count("(global_step=2)") == 2, out[-4000:]
    assert tb.latest_checkpoint(td).endswith("model.ckpt-4")
