"""Run-to-run determinism and checkpoint/resume continuity of the GPU engine
(SURVEY §4 "Resume: save, kill, resume, and require bit-identical state"; §5
race-detection row "run-to-run determinism test").

The step is deterministic by construction: split-K weight gradients are reduced
in a fixed order (wgrad_reduce_grouped), the BN statistics go through fp64
accumulators whose fp32 inputs sum exactly, the augmentation's RNG is keyed on
global_step, and the per-stream issue threads only change host timing, never the
device-side order of dependent work.  Reference flow: resnet_cifar_main.py:328-356
(MonitoredTrainingSession restores the latest checkpoint and continues)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from distributed_tensorflow_resnet_amd.models.spec import cifar_spec
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule
from distributed_tensorflow_resnet_amd.utils.checkpoint import Saver, state_to_tf

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIZE, N = 50, 32


def _engine(gpu):
    eng = Engine(cifar_spec(SIZE), N, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(),
                 device=gpu, seed=7, data_seed=99)
    eng.fill_synthetic(3)
    return eng


def _state(eng):
    torch.cuda.synchronize()
    return (eng.params.master.clone(), eng.mom.clone(), eng.params.stats.clone(),
            int(eng.gstep.item()))


def _same(a, b):
    return all(torch.equal(x, y) for x, y in zip(a[:3], b[:3])) and a[3] == b[3]


def test_same_seed_runs_are_bitwise_identical(gpu):
    runs = []
    for _ in range(2):
        eng = _engine(gpu)
        for _ in range(5):
            eng.step()
        runs.append(_state(eng))
        del eng
    assert _same(runs[0], runs[1])
    assert runs[0][3] == 5


_RESUME = r"""
import json, sys, torch
sys.path.insert(0, {root!r})
from distributed_tensorflow_resnet_amd.models.spec import cifar_spec
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule
from distributed_tensorflow_resnet_amd.utils.checkpoint import Saver, state_to_tf, tf_to_state
dev = torch.device("cuda", 0)
eng = Engine(cifar_spec({size}), {n}, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(),
             device=dev, seed=123, data_seed=99)   # different init: everything comes from the ckpt
eng.fill_synthetic(3)
saver = Saver({ckpt!r})
tf_to_state(Saver.restore(saver.latest()), eng.params, eng.mom, strict=True)
eng.sync_from_params()
for _ in range({steps}):
    eng.step()
torch.cuda.synchronize()
print(saver.save(state_to_tf(eng.params, eng.mom, int(eng.gstep.item())), int(eng.gstep.item())))
"""


def test_resume_in_fresh_process_is_bitwise_continuous(gpu, tmp_path):
    straight = _engine(gpu)
    for _ in range(40):
        straight.step()
    want = _state(straight)
    del straight

    half = _engine(gpu)
    for _ in range(20):
        half.step()
    torch.cuda.synchronize()
    ckpt = str(tmp_path / "train")
    saver = Saver(ckpt)
    saver.save(state_to_tf(half.params, half.mom, int(half.gstep.item())), 20)
    del half
    code = _RESUME.format(root=ROOT, size=SIZE, n=N, ckpt=ckpt, steps=20)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    got = Saver.restore(r.stdout.strip().splitlines()[-1])
    assert int(got["global_step"]) == 40
    ref = state_to_tf(*_fake_store(want, gpu), 40)
    bad = [k for k in ref if not np.array_equal(ref[k], got[k])]
    assert not bad, f"{len(bad)} tensors differ after resume, e.g. {bad[:4]}"


def _fake_store(state, gpu):
    """(ParamStore, momentum) holding a captured engine state, for state_to_tf."""
    from distributed_tensorflow_resnet_amd.models.params import ParamStore

    store = ParamStore(cifar_spec(SIZE), device=gpu)
    store.master.copy_(state[0])
    store.stats.copy_(state[2])
    return store, state[1]
