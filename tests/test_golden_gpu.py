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

REF_PB = "/root/reference/test/resnet50-cifar-ckpt-20190218/resnet50_cifar_frozen_model_eval.pb"
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


def test_full_depth_training_step_from_trained_weights(gpu, trained):
    """CIFAR ResNet-50 (full depth, training-mode BN): per-tensor gradients of one
    engine step vs fp32 autograd of the same TF-semantics network."""
    spec = cifar_spec(50)
    N = 64
    eng = Engine(spec, N, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(), device=gpu,
                 input_mode="nhwc", use_graph=False)
    tf_to_state(trained, eng.params, None, strict=True)
    eng.repack()
    torch.manual_seed(1)
    imgs = torch.randn(N, 32, 32, 3, device=gpu).to(torch.bfloat16).float()
    labels = torch.randint(0, 10, (N,), device=gpu)
    eng.set_batch(imgs, labels)
    st = torch.cuda.current_stream().cuda_stream
    eng._run("fwd", st)
    eng._run("bwd", st)
    torch.cuda.synchronize()

    store = ParamStore(spec, device=gpu)
    tf_to_state(trained, store, None, strict=True)
    model = TorchResNet(spec, store)
    logits = model(imgs, True)
    xent, _ = model.loss(logits, labels, 2e-4)
    xent.backward()
    g_ref = store.master.grad.detach()
    assert abs(eng.scalars[0].item() / N - xent.item()) < 1e-2 * max(1.0, xent.item())
    worst = sorted(((_rel(eng.grad[s.offset:s.offset + s.numel],
                          g_ref[s.offset:s.offset + s.numel]), s.name)
                    for s in eng.params.train_slots), reverse=True)
    glob = _rel(eng.grad, g_ref)
    print("global grad rel err", glob, "worst tensors", worst[:4])
    assert glob < 5e-2, worst[:5]
    assert worst[0][0] < 0.15, worst[:5]   # every tensor, including the first conv
    # BN moving statistics: one step of decay 0.997 towards the batch (Bessel) stats
    assert _rel(eng.params.stats, store.stats) < 1e-4
