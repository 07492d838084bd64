"""The GPU engine against the reference's own trained CIFAR-10 ResNet-50
(`resnet50_cifar_frozen_model_eval.pb`, decoded data-only; see
tests/test_graphdef_cpu.py).  Trained weights make the full-depth network
well conditioned, so these checks are tight where the random-init deep tests
in test_engine_gpu.py can only bound bf16 chaos."""
import os

import pytest
import torch

from distributed_tensorflow_resnet_amd.models.params import ParamStore
from distributed_tensorflow_resnet_amd.models.resnet_torch import TorchResNet
from distributed_tensorflow_resnet_amd.models.spec import cifar_spec
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule
from distributed_tensorflow_resnet_amd.utils import frozen
from distributed_tensorflow_resnet_amd.utils import graphdef as gd
from distributed_tensorflow_resnet_amd.utils.checkpoint import tf_to_state
from distributed_tensorflow_resnet_amd.utils.tf_interp import Interpreter

_HERE = os.path.dirname(os.path.abspath(__file__))
REF_PB = "/root/reference/test/resnet50-cifar-ckpt-20190218/resnet50_cifar_frozen_model_eval.pb"
if not os.path.exists(REF_PB):   # the GPU box sees only this repo: the fixture copy
    REF_PB = os.path.join(_HERE, "fixtures", "resnet50_cifar_frozen_model_eval.pb")
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not os.path.exists(REF_PB), reason="reference .pb absent")]


def _rel(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


@pytest.fixture(scope="module")
def trained():
    return frozen.read_frozen(REF_PB)[1]


def test_gpu_inference_matches_reference_graph(gpu, trained):
    """GPU eval plan (bf16 MFMA, moving-average BN) vs TF's graph run in fp64."""
    torch.manual_seed(0)
    n = 64
    x = torch.randn(n, 32, 32, 3).to(torch.bfloat16).float()
    labels = torch.randint(0, 10, (n,))
    y = torch.nn.functional.one_hot(labels, 10).float()
    probs_ref, logits_ref = Interpreter(gd.read_graph(REF_PB)).run(["Softmax", "final_dense"],
                                                                  {"X": x, "Y": y})
    m = frozen.FrozenModel(REF_PB, "gpu", n)
    probs, prec = m.predict(x, labels)
    err = _rel(probs, probs_ref)
    print(f"softmax rel err {err:.2e}")
    assert err < 2e-2
    agree = (probs.argmax(1) == probs_ref.argmax(1)).float().mean().item()
    assert agree >= 0.95, agree


@pytest.mark.parametrize("N", [64, 128])
def test_full_depth_training_step_from_trained_weights(gpu, trained, N, monkeypatch):
    """CIFAR ResNet-50 (full depth, training-mode BN) from the trained weights:
    one engine step's gradients vs fp32 autograd of the same TF-semantics network.

    Measured property of this network (scripts: bf16-emulating TorchResNet on the
    CPU): storing activations and gradients in bf16 -- as ANY bf16 trainer does --
    moves the full-depth gradient ~17 % from fp32 (the dense layer 2 %, the last
    conv 5 %, growing towards the stem), so a flat 5e-2 bound on every tensor is
    unattainable by a bf16 implementation.  What is pinned instead: the loss, the
    head's gradients tightly, the engine no noisier than the plain bf16 emulation,
    and the gradient direction.  N = 128 is the 1-GPU headline's kernel instance
    (bench.py): auto selection must pick the persistent step at one slice per image in
    both launches."""
    spec = cifar_spec(50)
    eng = Engine(spec, N, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(), device=gpu,
                 input_mode="nhwc", use_graph=False)
    if N == 128:
        assert eng.persist and (eng.prn.P, eng.prn.P_fwd) == (1, 1), eng.persist_reason
    tf_to_state(trained, eng.params, None, strict=True)
    eng.repack()
    torch.manual_seed(1)
    imgs = torch.randn(N, 32, 32, 3, device=gpu).to(torch.bfloat16).float()
    labels = torch.randint(0, 10, (N,), device=gpu)
    eng.set_batch(imgs, labels)
    st = torch.cuda.current_stream().cuda_stream
    eng.forward_backward(st)
    torch.cuda.synchronize()

    ref = {}
    for emu in (False, True):
        store = ParamStore(spec, device=gpu)
        tf_to_state(trained, store, None, strict=True)
        model = TorchResNet(spec, store, emulate_bf16=emu)
        logits = model(imgs, True)
        xent, _ = model.loss(logits, labels, 2e-4)
        xent.backward()
        ref[emu] = (xent, store.master.grad.detach(), store)
    xent, g32, store = ref[False]
    g_emu = ref[True][1]
    sl = {s.name: slice(s.offset, s.offset + s.numel) for s in eng.params.train_slots}
    err, noise = _rel(eng.grad, g32), _rel(g_emu, g32)
    cos = torch.nn.functional.cosine_similarity(eng.grad.double(), g32.double(), dim=0).item()
    per = {n: _rel(eng.grad[sl[n]], g32[sl[n]]) for n in sl}
    print(f"engine vs fp32 {err:.3f} (cos {cos:.4f}); bf16-emulation vs fp32 {noise:.3f}; "
          f"dense {per['dense/kernel']:.3f}/{per['dense/bias']:.3f} last conv "
          f"{per['conv2d_51/kernel']:.3f}")
    assert abs(eng.scalars[0].item() / N - xent.item()) < 1e-2 * max(1.0, xent.item())
    assert per["dense/kernel"] < 5e-2 and per["dense/bias"] < 5e-2
    assert per["conv2d_51/kernel"] < 0.1
    assert err <= 1.15 * noise + 1e-3, (err, noise)
    assert cos > 0.98
    # per stage (stem, the three block layers): a regression confined to the early
    # layers must not hide behind the global bound
    def stage(name):
        base = name.split("/")[0]
        if base.startswith("conv2d"):
            i = int(base.split("_")[1]) if "_" in base else 0
            return "stem" if i == 0 else f"stage{(i - 1) // 17 + 1}"
        if base.startswith("batch_normalization"):
            i = int(base.split("_")[2]) if base.count("_") == 2 else 0
            return f"stage{i // 16 + 1}" if i < 48 else "head"
        return "head"
    groups = {}
    for n, s_ in sl.items():
        groups.setdefault(stage(n), []).append(s_)
    for gname in ("stem", "stage1", "stage2", "stage3"):
        idx = torch.cat([torch.arange(s_.start, s_.stop, device=gpu) for s_ in groups[gname]])
        e_s, n_s = _rel(eng.grad[idx], g32[idx]), _rel(g_emu[idx], g32[idx])
        print(f"{gname}: engine {e_s:.3f} vs bf16-emulation {n_s:.3f}")
        assert e_s <= 1.15 * n_s + 1e-3, (gname, e_s, n_s)
    # BN moving statistics: one step of decay 0.997 towards the batch (Bessel) stats
    assert _rel(eng.params.stats, store.stats) < 1e-4
    if N == 128:
        # the headline instance against the launch-per-layer engine, stage by stage
        monkeypatch.setenv("DTR_TUNE", "persist=0")
        er = Engine(spec, N, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(), device=gpu,
                    input_mode="nhwc", use_graph=False)
        assert not er.persist
        tf_to_state(trained, er.params, None, strict=True)
        er.repack()
        er.set_batch(imgs, labels)
        er.forward_backward(st)
        torch.cuda.synchronize()
        for gname in ("stem", "stage1", "stage2", "stage3", "head"):
            idx = torch.cat([torch.arange(s_.start, s_.stop, device=gpu) for s_ in groups[gname]])
            c = torch.nn.functional.cosine_similarity(eng.grad[idx].double(), er.grad[idx].double(),
                                                      dim=0).item()
            e_p, e_l = _rel(eng.grad[idx], g32[idx]), _rel(er.grad[idx], g32[idx])
            print(f"{gname}: persistent-vs-per-layer cos {c:.4f}; vs fp32 {e_p:.3f} / {e_l:.3f}")
            assert c > 0.98, (gname, c)
            assert e_p <= 1.15 * e_l + 1e-2, (gname, e_p, e_l)
        assert _rel(eng.params.stats, er.params.stats) < 1e-4
