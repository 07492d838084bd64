"""Persistent small-batch CIFAR step (csrc/cifar_persist.hip, train/persist.py) against
the launch-per-layer engine and the fp32 autograd oracle of the same network."""
import pytest
import torch

from distributed_tensorflow_resnet_amd.models.params import ParamStore
from distributed_tensorflow_resnet_amd.models.resnet_torch import TorchResNet
from distributed_tensorflow_resnet_amd.models.spec import cifar_spec
from distributed_tensorflow_resnet_amd.train.engine import Engine, cifar_lr_schedule

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _engine(monkeypatch, spec, N, gpu, persist, input_mode="nhwc", slices=-1, opt_fused=1):
    monkeypatch.setenv("DTR_TUNE", f"persist={persist},persist_slices={slices},opt_fused={opt_fused}")
    eng = Engine(spec, N, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(), device=gpu,
                 input_mode=input_mode, use_graph=False)
    assert eng.persist == (persist == 1)
    return eng


def _batch(spec, N, gpu, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    imgs = torch.randn(N, spec.image_h, spec.image_w, 3, generator=g).to(torch.bfloat16).float()
    labels = torch.randint(0, spec.num_classes, (N,), generator=g)
    return imgs.to(gpu), labels.to(gpu)


def _pair(monkeypatch, spec, N, gpu, slices=-1):
    ep = _engine(monkeypatch, spec, N, gpu, 1, slices=slices)
    er = _engine(monkeypatch, spec, N, gpu, 0)
    er.params.master.copy_(ep.params.master)
    er.params.stats.copy_(ep.params.stats)
    er.repack()
    imgs, labels = _batch(spec, N, gpu)
    for e in (ep, er):
        e.set_batch(imgs, labels)
    return ep, er, imgs, labels


@pytest.mark.parametrize("size,N,slices", [(8, 16, 4), (20, 32, 2), (50, 16, 4), (20, 16, 1),
                                           (8, 64, 2), (8, 40, 4), (8, 112, 2)])
def test_persistent_forward_matches_per_layer(gpu, monkeypatch, size, N, slices):
    """Saved activations, batch statistics and head outputs of the one-launch forward
    vs the per-layer forward (same weights, same batch): bf16-rounding agreement, for
    4, 2 and 1 row slices per image."""
    spec = cifar_spec(size)
    ep, er, _, _ = _pair(monkeypatch, spec, N, gpu, slices)
    assert ep.prn.P == slices
    st = torch.cuda.current_stream().cuda_stream
    for e in (ep, er):
        e._run("fwd", st)
    torch.cuda.synchronize()
    assert not ep.persist_error()
    worst = 0.0
    for i in range(len(spec.blocks)):
        for a, b in ((ep.X[i + 1], er.X[i + 1]), (ep.H1[i], er.H1[i])):
            worst = max(worst, _rel(a, b))
    assert _rel(ep.X[0], er.X[0]) < 1e-2
    assert worst < 5e-2, worst
    for name, bp in ep.bns.items():
        br = er.bns[name]
        assert _rel(bp.mean, br.mean) < 5e-2 + 1e-3 * br.mean.abs().max().item(), name
        assert _rel(bp.rstd, br.rstd) < 2e-2, name
    assert _rel(ep.pooled, er.pooled) < 3e-2
    assert _rel(ep.dlogits.float(), er.dlogits.float()) < 3e-2
    assert _rel(ep.params.stats, er.params.stats) < 1e-3   # moving averages


@pytest.mark.parametrize("size,N,slices", [(8, 16, 4), (8, 32, 2), (8, 16, 1), (8, 48, 2),
                                           (8, 56, 4), (8, 96, 2)])
def test_persistent_step_matches_autograd(gpu, monkeypatch, size, N, slices):
    """Whole training step (forward + backward + slab reduces): per-tensor gradients
    vs the bf16-emulating fp32 oracle, like test_engine_step_matches_autograd_shallow."""
    spec = cifar_spec(size)
    ep = _engine(monkeypatch, spec, N, gpu, 1, slices=slices)
    assert ep.prn.P == slices
    imgs, labels = _batch(spec, N, gpu)
    ep.set_batch(imgs, labels)
    store = ParamStore(spec, device=gpu)
    store.master.copy_(ep.params.master)
    store.stats.copy_(ep.params.stats)
    st = torch.cuda.current_stream().cuda_stream
    ep.forward_backward(st)
    torch.cuda.synchronize()
    assert not ep.persist_error()
    model = TorchResNet(spec, store, emulate_bf16=True)
    logits = model(imgs, True)
    xent, _ = model.loss(logits, labels, 2e-4)
    xent.backward()
    g_ref = store.master.grad.detach()
    assert abs(ep.scalars[0].item() / N - xent.item()) < 1e-2 * max(1.0, xent.item())
    worst = sorted(((_rel(ep.grad[s.offset:s.offset + s.numel], g_ref[s.offset:s.offset + s.numel]),
                     s.name) for s in ep.params.train_slots), reverse=True)
    print("worst per-tensor gradient rel err:", worst[:4], "global", _rel(ep.grad, g_ref))
    assert _rel(ep.grad, g_ref) < 5e-2, worst[:5]
    assert _rel(ep.params.stats, store.stats) < 1e-3


@pytest.mark.parametrize("size,N", [(20, 32), (50, 16), (50, 32)])
def test_persistent_step_within_bf16_noise_deep(gpu, monkeypatch, size, N):
    """Deep random-init ResNets are chaotic under bf16 rounding (test_engine_gpu.py,
    test_engine_step_within_bf16_noise_deep): the persistent gradient must be at least
    as close to the bf16-emulating oracle as fp32 is, point the same way as the
    per-layer engine's, and every BatchNorm parameter gradient must be finite."""
    spec = cifar_spec(size)
    ep, er, imgs, labels = _pair(monkeypatch, spec, N, gpu)
    out = {}
    for emu in (True, False):
        store = ParamStore(spec, device=gpu)
        store.master.copy_(ep.params.master)
        store.stats.copy_(ep.params.stats)
        model = TorchResNet(spec, store, emulate_bf16=emu)
        xent, _ = model.loss(model(imgs, True), labels, 2e-4)
        xent.backward()
        out[emu] = (xent.item(), store.master.grad.detach().clone())
    st = torch.cuda.current_stream().cuda_stream
    for e in (ep, er):
        e.forward_backward(st)
    torch.cuda.synchronize()
    assert not ep.persist_error()
    (x_emu, g_emu), (_, g_32) = out[True], out[False]
    assert abs(ep.scalars[0].item() / N - x_emu) < 2e-2 * max(1.0, x_emu)
    noise = _rel(g_32, g_emu)
    err, err_layer = _rel(ep.grad, g_emu), _rel(er.grad, g_emu)
    cos = torch.nn.functional.cosine_similarity(ep.grad, er.grad, dim=0).item()
    print(f"persistent-vs-emu {err:.3f}, per-layer-vs-emu {err_layer:.3f}, fp32-vs-emu "
          f"{noise:.3f}; persistent-vs-per-layer cos {cos:.4f}")
    assert err <= max(0.05, noise), (err, noise)
    assert cos > 0.9
    assert torch.isfinite(ep.grad).all()


@pytest.mark.parametrize("size,N,slices", [(20, 16, 4), (20, 32, 2), (50, 128, 1),
                                           (8, 56, 4)])
def test_persistent_step_bitwise_under_concurrent_load(gpu, monkeypatch, size, N, slices):
    """Race stress for the hand-off protocol (write-through publishes, drained arrives,
    sc1 reads, the weight-gradient readiness line): while the persistent launches run,
    another stream keeps a CU busy (so one slice workgroup starts late and every other
    waits at the barriers) and streams memory-heavy kernels through the L2s.  Every run
    must reproduce the quiet run's gradient bit for bit and never time out.  RN50 at
    N = 128, one slice: the 1-GPU headline's kernel instance (bench.py)."""
    spec = cifar_spec(size)
    eng = _engine(monkeypatch, spec, N, gpu, 1, slices=slices)
    imgs, labels = _batch(spec, N, gpu)
    eng.set_batch(imgs, labels)
    st = torch.cuda.current_stream()
    eng.forward_backward(st.cuda_stream)
    torch.cuda.synchronize()
    ref = eng.grad.clone()
    noise = torch.cuda.Stream(device=gpu)
    big = torch.zeros(64 << 20, device=gpu)   # 256 MB
    for i in range(6):
        with torch.cuda.stream(noise):
            torch.cuda._sleep(20000 * (i + 1))   # one CU busy for ~10-60 us
            for _ in range(2):
                big.add_(1.0)
        eng.forward_backward(st.cuda_stream)
        torch.cuda.synchronize()
        assert not eng.persist_error()
        assert torch.equal(eng.grad, ref), f"run {i}: gradient differs under concurrent load"


@pytest.mark.parametrize("N", [16, 128])
def test_fused_optimizer_matches_unfused(gpu, monkeypatch, N):
    """opt_fused (ONE sgd_tiles launch: slab sums + SGD-momentum + both bf16 copies +
    global_step) vs the grouped reduce + sgd_pack + ohwi_pack launches
    from the same weights on the same batch: after one step the gradients are equal bit
    for bit (N = 128: 32-split slabs, summed in the grouped reduce's order), weights,
    momenta and the bf16 copies agree to fp32 rounding (the update's fma contraction),
    and the ticket re-arms (global_step counts every step)."""
    spec = cifar_spec(20)
    ef = _engine(monkeypatch, spec, N, gpu, 1, input_mode="cifar_u8", opt_fused=1)
    eu = _engine(monkeypatch, spec, N, gpu, 1, input_mode="cifar_u8", opt_fused=0)
    assert "gsum" in ef.seg and "gsum" not in eu.seg
    eu.params.master.copy_(ef.params.master)
    eu.params.stats.copy_(ef.params.stats)
    eu.repack()
    for e in (ef, eu):
        e.fill_synthetic(0)
    for e in (ef, eu):
        e.step()
    torch.cuda.synchronize()
    assert not ef.persist_error() and not eu.persist_error()
    mf, mu = ef.metrics(reduce=False), eu.metrics(reduce=False)
    assert mf["global_step"] == mu["global_step"] == 1
    assert mf["lr"] == mu["lr"]
    print("rel grad", _rel(ef.grad, eu.grad), "master", _rel(ef.params.master, eu.params.master),
          "mom", _rel(ef.mom, eu.mom), "wbf", _rel(ef.wbf, eu.wbf))
    assert torch.equal(ef.grad, eu.grad)   # the grouped reduce's summation order
    assert _rel(ef.params.master, eu.params.master) < 1e-6
    assert _rel(ef.mom, eu.mom) < 1e-5
    assert _rel(ef.wbf, eu.wbf) < 1e-3
    # (later steps drift apart: a deep bf16 network amplifies the last-bit differences of
    # the N = 128 slab sums) -- the step counter and the ticket keep counting
    for _ in range(2):
        ef.step()
    torch.cuda.synchronize()
    assert ef.metrics(reduce=False)["global_step"] == 3
    assert ef.opt_ticket.item() == 0
    assert torch.isfinite(ef.params.master).all()
