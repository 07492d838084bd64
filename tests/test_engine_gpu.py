"""End-to-end: one engine training step (native plan, bf16 MFMA kernels) against
the fp32 autograd execution of the same TF-semantics network (models/resnet_torch.py)."""
import copy

import pytest
import torch

from distributed_tensorflow_resnet_amd.models.params import ParamStore
from distributed_tensorflow_resnet_amd.models.resnet_torch import TorchResNet
from distributed_tensorflow_resnet_amd.models.spec import cifar_spec, imagenet_spec
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _per_layer_engine(monkeypatch):
    """These tests pin the launch-per-layer engine and its knobs (the persistent CIFAR
    step, the default for CIFAR batches <= 240, is covered by test_persist_gpu.py)."""
    monkeypatch.setenv("DTR_TUNE", "persist=0")


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _make(spec, N, gpu, wd=2e-4):
    eng = Engine(spec, N, weight_decay=wd, lr_schedule=cifar_lr_schedule(), device=gpu,
                 input_mode="nhwc", use_graph=False)
    torch.manual_seed(0)
    imgs = torch.randn(N, spec.image_h, spec.image_w, 3, device=gpu).to(torch.bfloat16).float()
    labels = torch.randint(0, spec.num_classes, (N,), device=gpu)
    eng.set_batch(imgs, labels)
    ref_store = ParamStore(spec, device=gpu)
    ref_store.master.copy_(eng.params.master)
    ref_store.stats.copy_(eng.params.stats)
    return eng, imgs, labels, ref_store


def _grads(spec, N, gpu):
    eng, imgs, labels, ref_store = _make(spec, N, gpu)
    st = torch.cuda.current_stream().cuda_stream
    eng.forward_backward(st)
    torch.cuda.synchronize()
    out = {}
    for emu in (True, False):
        store = ParamStore(spec, device=gpu)
        store.master.copy_(ref_store.master)
        store.stats.copy_(ref_store.stats)
        model = TorchResNet(spec, store, emulate_bf16=emu)
        logits = model(imgs, True)
        xent, _ = model.loss(logits, labels, 2e-4)
        xent.backward()
        out[emu] = (xent.item(), store.master.grad.detach().clone(), store)
    return eng, out


SHALLOW = [
    (lambda: cifar_spec(8), 16),
    (lambda: cifar_spec(8), 64),
]


@pytest.mark.parametrize("spec_fn,N", SHALLOW)
def test_engine_step_matches_autograd_shallow(gpu, spec_fn, N):
    """Well-conditioned nets: per-tensor gradients vs the bf16-emulating oracle."""
    spec = spec_fn()
    eng, out = _grads(spec, N, gpu)
    xent, g_ref, store = out[True]
    assert abs(eng.scalars[0].item() / N - xent) < 1e-2 * max(1.0, xent)
    worst = sorted(((_rel(eng.grad[s.offset:s.offset + s.numel],
                          g_ref[s.offset:s.offset + s.numel]), s.name)
                    for s in eng.params.train_slots), reverse=True)
    print("worst per-tensor gradient rel err:", worst[:4], "global", _rel(eng.grad, g_ref))
    assert _rel(eng.grad, g_ref) < 5e-2, worst[:5]
    # BN moving statistics updated like TF (decay 0.997, Bessel variance)
    assert _rel(eng.params.stats, store.stats) < 1e-3


@pytest.mark.parametrize("spec_fn,N", [
    (lambda: cifar_spec(20), 32),
    (lambda: imagenet_spec(18, image_hw=64), 8),
    (lambda: imagenet_spec(50, image_hw=64), 8),
    # ImageNet stem + max-pool: argmax flips make even shallow nets noisy
    (lambda: imagenet_spec(0, image_hw=64, block="bottleneck", layers=[1, 1, 1, 1]), 8),
    (lambda: imagenet_spec(0, image_hw=64, block="building", layers=[1, 1, 1, 1]), 8),
])
def test_engine_step_within_bf16_noise_deep(gpu, spec_fn, N):
    """Deep random-init ResNets are chaotic under bf16 rounding (fp32 and the
    bf16-emulating oracle themselves disagree by 30-110%): require the engine to
    be at least as close to the emulating oracle as fp32 is."""
    spec = spec_fn()
    eng, out = _grads(spec, N, gpu)
    (x_emu, g_emu, _), (x_32, g_32, _) = out[True], out[False]
    assert abs(eng.scalars[0].item() / N - x_emu) < 2e-2 * max(1.0, x_emu)
    noise = _rel(g_32, g_emu)
    err = _rel(eng.grad, g_emu)
    cos_e = torch.nn.functional.cosine_similarity(eng.grad, g_emu, dim=0).item()
    cos_32 = torch.nn.functional.cosine_similarity(g_32, g_emu, dim=0).item()
    print(f"engine-vs-emu {err:.3f} (cos {cos_e:.3f}); fp32-vs-emu {noise:.3f} (cos {cos_32:.3f})")
    assert err <= max(0.05, noise), (err, noise)
    assert cos_e >= cos_32 - 0.05


def test_optimizer_step_and_pack(gpu, monkeypatch):
    """SGD-momentum + weight decay and the bf16 weight copies, by sgd_pack + ohwi_pack
    (the launch-per-layer plan; the persistent step's one-launch sgd_tiles:
    test_persist_gpu.py)."""
    monkeypatch.setenv("DTR_TUNE", "persist=0")
    spec = cifar_spec(8)
    eng, imgs, labels, _ = _make(spec, 16, gpu)
    w0 = eng.params.master.clone()
    eng.step()
    torch.cuda.synchronize()
    g = eng.grad
    lr = 0.1  # step 0 uses the hook's begin() value
    expect = w0 - lr * (g + 2e-4 * w0)
    torch.testing.assert_close(eng.params.master, expect, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(eng.mom, g + 2e-4 * w0, rtol=1e-5, atol=1e-7)
    assert int(eng.gstep.item()) == 1
    m = eng.metrics()
    assert abs(m["lr"] - 0.1) < 1e-7
    # bf16 copies track the master (forward OHWI layout of conv2d_2)
    c = eng.convs["conv2d_2"]
    s = eng.params.slot("conv2d_2/kernel")
    w = eng.params.master[s.offset:s.offset + s.numel].view(s.shape)  # HWIO
    n = w.numel()
    off = (c.ohwi - eng.wbf.data_ptr()) // 2
    ohwi = eng.wbf[off:off + n].view(s.shape[3], s.shape[0], s.shape[1], s.shape[2])
    torch.testing.assert_close(ohwi.float(), w.permute(3, 0, 1, 2).to(torch.bfloat16).float())


@pytest.mark.parametrize("persist", [0, 1])
def test_graph_replay_matches_eager(gpu, monkeypatch, persist):
    """(persist: the persistent step, whose one-launch optimizer's global_step ticket
    re-arms across graph replays)"""
    monkeypatch.setenv("DTR_TUNE", f"persist={persist}")
    spec = cifar_spec(8)
    e1, imgs, labels, _ = _make(spec, 16, gpu)
    e2 = Engine(spec, 16, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(), device=gpu,
                input_mode="nhwc")
    e2.params.master.copy_(e1.params.master)
    e2.params.stats.copy_(e1.params.stats)
    e2.repack()
    e2.set_batch(imgs, labels)
    for _ in range(4):
        e1.step()
    e2.capture(warmup=2)
    e2.step()
    e2.step()
    torch.cuda.synchronize()
    assert int(e2.gstep.item()) == 4
    torch.testing.assert_close(e1.params.master, e2.params.master, rtol=0, atol=0)


def test_training_reduces_loss(gpu):
    spec = cifar_spec(20)
    eng = Engine(spec, 64, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(), device=gpu)
    eng.fill_synthetic(0)
    eng.capture(warmup=2)
    first = None
    for i in range(60):
        eng.step()
        if i == 0:
            first = eng.metrics()["cross_entropy"]
    last = eng.metrics()["cross_entropy"]
    assert last < first * 0.7, (first, last)


def test_eval_plan_matches_autograd_eval(gpu):
    spec = cifar_spec(8)
    eng, imgs, labels, ref_store = _make(spec, 16, gpu)
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    ref_store.master.copy_(eng.params.master)
    ref_store.stats.copy_(eng.params.stats)
    ev = eng.build_eval_plan(8)
    loss_sum, correct, probs = ev.run(imgs[:8], labels[:8], raw_u8=False)
    model = TorchResNet(spec, ref_store)
    with torch.no_grad():
        logits = model(imgs[:8], False)
    p_ref = torch.softmax(logits, 1)
    assert _rel(probs, p_ref) < 2e-2


def test_bn_accumulator_mode_matches_partials(gpu, monkeypatch):
    """tune bn_acc=1 (fp64 atomic accumulators per BatchNorm) vs the per-tile partial
    path: same loss, gradients and BN statistics up to rounding (shallow net; deep
    nets are chaotic under bf16 and covered by the oracle tests above)."""
    spec = cifar_spec(8)
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("DTR_TUNE", f"bn_acc={mode},persist=0")
        eng, _, _, _ = _make(spec, 64, gpu)
        st = torch.cuda.current_stream().cuda_stream
        eng.forward_backward(st)
        torch.cuda.synchronize()
        res[mode] = (eng.scalars[0].item(), eng.grad.clone(), eng.params.stats.clone())
    (l0, g0, s0), (l1, g1, s1) = res["0"], res["1"]
    assert abs(l1 - l0) <= 1e-4 * max(1.0, abs(l0))
    assert _rel(g1, g0) < 1e-2
    assert _rel(s1, s0) < 1e-5


def test_fused_head_matches_unfused(gpu, monkeypatch):
    """head_fused (one launch: final BN finalize .. final BN backward sums) vs the
    8-launch head: same loss, precision, gradients and BN statistics up to rounding."""
    spec = cifar_spec(8)
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("DTR_TUNE", f"fused_head={mode},persist=0")
        eng, _, _, _ = _make(spec, 64, gpu)
        assert eng._head_fused == (mode == "1")
        st = torch.cuda.current_stream().cuda_stream
        eng.forward_backward(st)
        torch.cuda.synchronize()
        res[mode] = (eng.scalars[:2].clone(), eng.grad.clone(), eng.params.stats.clone())
    (s0, g0, t0), (s1, g1, t1) = res["0"], res["1"]
    assert abs(s1[0].item() - s0[0].item()) <= 1e-4 * max(1.0, abs(s0[0].item()))
    assert s1[1].item() == s0[1].item()
    assert _rel(g1, g0) < 1e-2
    assert _rel(t1, t0) < 1e-5


def test_bn_backward_apply_recompute_matches_separate_apply(gpu, monkeypatch):
    """tune bap_maxc: the identity bottleneck blocks' first 1x1 dgrad runs twice (BN-backward
    sums, then BN+ReLU backward + the residual gradient applied in the second pass) instead of
    dgrad + BN-backward sums + a separate apply.  Both use the streaming kernel
    (bn_dgrad1x1.hip) with the same tile order for the sums, and the apply arithmetic is the
    separate apply's, so the whole step is bitwise equal."""
    spec = imagenet_spec(50, image_hw=64)
    res = {}
    for mode in ("0", "2048"):
        monkeypatch.setenv("DTR_TUNE", f"bap_maxc={mode},persist=0")
        eng, _, _, _ = _make(spec, 8, gpu)
        st = torch.cuda.current_stream().cuda_stream
        eng.forward_backward(st)
        torch.cuda.synchronize()
        res[mode] = (eng.scalars[0].item(), eng.grad.clone(), eng.params.stats.clone(),
                     eng.n_bap)
    (l0, g0, s0, n0), (l1, g1, s1, n1) = res["0"], res["2048"]
    assert (n0, n1) == (0, 12)   # RN50: 3 + 4 + 6 + 3 blocks, one projection block each
    assert l1 == l0
    assert torch.equal(s1, s0)
    assert torch.equal(g1, g0)


def test_streaming_fwd1x1_matches_implicit_gemm(gpu, monkeypatch):
    """tune fwd1x1_stream: the expanding 1x1 convs (and the stage-1 projection) on the
    streaming kernel vs the implicit-GEMM tile.  Per conv the outputs are bitwise equal
    (test_streaming_narrow_fwd_bn_residual_stats); through the network the BN statistics'
    summation order differs (fp64 sums, 1e-8 relative), which bf16 rounding flips amplify
    block by block: the forward agrees to bf16 noise.  (At random init the backward is
    ill-conditioned -- saturated softmax -- so gradients are compared against the fp32
    oracle instead: test_engine_step_within_bf16_noise_deep runs this default path.)"""
    spec = imagenet_spec(0, image_hw=64, block="bottleneck", layers=[2, 2, 2, 2])
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("DTR_TUNE", f"fwd1x1_stream={mode},persist=0")
        eng, _, _, _ = _make(spec, 8, gpu)
        st = torch.cuda.current_stream().cuda_stream
        eng._run("fwd", st)
        torch.cuda.synchronize()
        res[mode] = (eng.scalars[0].item(), [x.float().clone() for x in eng.X],
                     eng.params.stats.clone())
    (l0, x0, s0), (l1, x1, s1) = res["0"], res["1"]
    assert abs(l1 - l0) <= 5e-3 * max(1.0, abs(l0))
    rels = [_rel(b, a) for a, b in zip(x0, x1)]
    assert rels[0] == 0.0 and all(r < 5e-2 for r in rels), rels
    assert _rel(s1, s0) < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("spec_fn,N,fork_every", [
    (lambda: cifar_spec(50), 16, "2"),
    (lambda: cifar_spec(20), 32, "1"),
    (lambda: imagenet_spec(18), 8, "2"),
])
def test_built_plans_pass_stream_order_check(gpu, monkeypatch, spec_fn, N, fork_every):
    """The engine refuses a plan with a fork/join race at construction
    (utils/streamcheck.py); pin that real plans are checked and pass, and that the
    check sees side-stream work at all (otherwise it would pass vacuously)."""
    from distributed_tensorflow_resnet_amd.utils.streamcheck import check_plan

    monkeypatch.setenv("DTR_TUNE", f"fork_every={fork_every},persist=0")
    eng = Engine(spec_fn(), N, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(),
                 device=gpu, use_graph=False)
    assert eng.fork_wgrad
    assert check_plan(eng.plan, eng.seg) == []
    a, b = eng.seg["bwd"]
    assert 1 in eng.plan.op_streams()[a:b]
    assert 2 in eng.plan.op_kinds()[a:b]
