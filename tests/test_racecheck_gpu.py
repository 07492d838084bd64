"""Schedule-perturbation race check (utils/racecheck.py, Plan.set_perturb).

First the checker is shown to catch the two race shapes the static fork/join
check cannot see by buffer (a missing join: main reads what the side stream is
still writing; a missing fork: the side stream reads what main has not written
yet).  Then the real training steps, CIFAR and ImageNet, must give the same
state bit for bit under every perturbed schedule as in plan order on one stream."""
import pytest
import torch

from distributed_tensorflow_resnet_amd.utils.racecheck import _make_factory, perturbation_check

pytestmark = pytest.mark.gpu


def _run(p, mode, seed=0):
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    p.set_perturb(mode, seed, 1.0, 200.0)
    p.run(0, p.size(), torch.cuda.current_stream().cuda_stream, s1.cuda_stream, s2.cuda_stream)
    torch.cuda.synchronize()


def _racy_plan(nat, x, b, c, n, join):
    """main: fork -> side: b = bf16(x); [join] -> main: c = f32(b)."""
    p = nat.Plan()
    e = p.new_event()
    p.record(e)
    p.use_stream(1)
    p.wait(e)
    p.cast_f32_bf16(x.data_ptr(), b.data_ptr(), n)
    if join:
        e2 = p.new_event()
        p.record(e2)
    p.use_stream(0)
    if join:
        p.wait(e2)
    p.cast_bf16_f32(b.data_ptr(), c.data_ptr(), n)
    return p


def _unforked_plan(nat, x, b, c, n):
    """main: b = bf16(x); side (no fork): c = f32(b); joined at the end."""
    p = nat.Plan()
    p.cast_f32_bf16(x.data_ptr(), b.data_ptr(), n)
    p.use_stream(1)
    p.cast_bf16_f32(b.data_ptr(), c.data_ptr(), n)
    e = p.new_event()
    p.record(e)
    p.use_stream(0)
    p.wait(e)
    return p


@pytest.mark.parametrize("shape", ["missing_join", "missing_fork"])
def test_perturbation_exposes_races(gpu, shape):
    import distributed_tensorflow_resnet_amd as dtr

    nat = dtr.native(required=True)
    n = 1 << 22
    x = torch.rand(n, device=gpu) + 1.0
    b = torch.zeros(n, dtype=torch.bfloat16, device=gpu)
    c = torch.zeros(n, device=gpu)
    p = (_racy_plan(nat, x, b, c, n, join=False) if shape == "missing_join"
         else _unforked_plan(nat, x, b, c, n))
    want = x.to(torch.bfloat16).float()
    _run(p, 1)
    assert torch.equal(c, want)          # plan order on one stream is the program's meaning
    caught = 0
    for t in range(6):
        b.zero_()
        c.zero_()
        torch.cuda.synchronize()
        _run(p, 2, seed=t)
        caught += not torch.equal(c, want)
    assert caught > 0, "no perturbed schedule exposed the race"


def test_perturbation_passes_joined_plan(gpu):
    import distributed_tensorflow_resnet_amd as dtr

    nat = dtr.native(required=True)
    n = 1 << 22
    x = torch.rand(n, device=gpu) + 1.0
    b = torch.zeros(n, dtype=torch.bfloat16, device=gpu)
    c = torch.zeros(n, device=gpu)
    p = _racy_plan(nat, x, b, c, n, join=True)
    want = x.to(torch.bfloat16).float()
    for t in range(6):
        b.zero_()
        c.zero_()
        torch.cuda.synchronize()
        _run(p, 2, seed=t)
        assert torch.equal(c, want), t


@pytest.mark.parametrize("model,batch", [("cifar_resnet50", 16), ("imagenet_resnet50", 4)])
def test_training_step_is_schedule_independent(gpu, model, batch):
    res = perturbation_check(_make_factory(model, batch, gpu), steps=3, trials=3, prob=0.3,
                             max_us=20.0)
    print(res)
    assert res["ok"], res["mismatches"]
