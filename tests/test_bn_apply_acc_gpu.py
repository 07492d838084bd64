"""bn_relu_apply_acc (csrc/bn.hip): the accumulator-mode BatchNorm finalize fused into
the materializing BN+ReLU pass equals bn_finalize (acc) + bn_relu_apply bitwise, and
both match an fp32 PyTorch batch-norm + ReLU of the same tensor (FusedBatchNorm
training mode, resnet_model_official.py:48-55: biased batch variance for the
normalization, Bessel-corrected variance in the moving average)."""
import pytest
import torch

from distributed_tensorflow_resnet_amd import native

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,C", [(25088, 256), (6272, 512), (1000, 64)])
def test_bn_relu_apply_acc_equals_finalize_then_apply(gpu, M, C):
    nat = native(required=True)
    rep = nat.bn_acc_rep()
    torch.manual_seed(0)
    x = (torch.randn(M, C, device=gpu) * 2 + 0.5).to(torch.bfloat16)
    xf = x.float().double()
    # fp64 replicas as the producing conv leaves them: sum y, sum y^2 split over replicas
    acc = torch.zeros(rep, 2, C, dtype=torch.float64, device=gpu)
    for r in range(rep):
        part = xf[r::rep]
        acc[r, 0] = part.sum(0)
        acc[r, 1] = (part * part).sum(0)
    gamma = torch.rand(C, device=gpu) + 0.5
    beta = torch.randn(C, device=gpu) * 0.1
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    for fused in (True, False):
        mm, mv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
        stats = [torch.empty(C, device=gpu) for _ in range(4)]   # mean, rstd, scale, shift
        y = torch.empty_like(x)
        p = [t.data_ptr() for t in stats]
        if fused:
            nat.bn_relu_apply_acc(x.data_ptr(), y.data_ptr(), M, C, acc.data_ptr(),
                                  gamma.data_ptr(), beta.data_ptr(), mm.data_ptr(), mv.data_ptr(),
                                  0.997, 1.001e-5, 1, *p, st)
        else:
            nat.bn_finalize(acc.data_ptr(), -1, 0, M, C, gamma.data_ptr(), beta.data_ptr(),
                            mm.data_ptr(), mv.data_ptr(), 0.997, 1.001e-5, 1, *p, st)
            nat.bn_relu_apply(x.data_ptr(), stats[2].data_ptr(), stats[3].data_ptr(),
                              y.data_ptr(), M, C, st)
        torch.cuda.synchronize()
        outs.append((y, mm, mv, stats))
    (y1, mm1, mv1, s1), (y2, mm2, mv2, s2) = outs
    assert torch.equal(y1, y2)
    assert torch.equal(mm1, mm2) and torch.equal(mv1, mv2)
    for a, b in zip(s1, s2):
        assert torch.equal(a, b)
    # fp32 reference
    xr = x.float()
    mu, var = xr.mean(0), xr.var(0, unbiased=False)
    ref = torch.relu((xr - mu) / torch.sqrt(var + 1.001e-5) * gamma + beta)
    assert ((y1.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2
    torch.testing.assert_close(mm1, 0.003 * mu, rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(mv1, 0.997 + 0.003 * xr.var(0, unbiased=True), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("M,C,add", [(25088, 1024, True), (100352, 512, False),
                                     (401408, 256, True), (4096, 64, False)])
def test_bn_bwd_apply_acc_equals_finalize_then_apply(gpu, M, C, add):
    """The BN+ReLU backward apply with the accumulator finalize fused in (any C the
    grid rule admits) equals bn_bwd_finalize (acc) + bn_bwd_apply bitwise."""
    nat = native(required=True)
    if not nat.bn_bwd_apply_acc_fits(M, C):
        pytest.skip("grid rule keeps this shape on the separate finalize")
    rep = nat.bn_acc_rep()
    torch.manual_seed(1)
    dy = torch.randn(M, C, device=gpu).to(torch.bfloat16)
    x = torch.randn(M, C, device=gpu).to(torch.bfloat16)
    ad = torch.randn(M, C, device=gpu).to(torch.bfloat16) if add else None
    acc = torch.randn(rep, 2, C, dtype=torch.float64, device=gpu) * 100
    mean, rstd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    scale, shift = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu) * 0.1
    gamma = torch.rand(C, device=gpu) + 0.5
    st = torch.cuda.current_stream().cuda_stream
    pa = 0 if ad is None else ad.data_ptr()
    res = []
    for fused in (True, False):
        dg, db, coef = (torch.zeros(C, device=gpu), torch.zeros(C, device=gpu),
                        torch.zeros(3 * C, device=gpu))
        dx = torch.empty_like(dy)
        if fused:
            nat.bn_bwd_apply_acc(dy.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                 scale.data_ptr(), shift.data_ptr(),
                                 [acc.data_ptr(), gamma.data_ptr(), dg.data_ptr(), db.data_ptr(),
                                  coef.data_ptr()], pa, dx.data_ptr(), M, C, st)
        else:
            nat.bn_bwd_finalize(acc.data_ptr(), -1, M, C, gamma.data_ptr(), rstd.data_ptr(),
                                dg.data_ptr(), db.data_ptr(), coef.data_ptr(), st)
            nat.bn_bwd_apply(dy.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                             scale.data_ptr(), shift.data_ptr(), coef.data_ptr(), pa,
                             dx.data_ptr(), M, C, st)
        torch.cuda.synchronize()
        res.append((dx, dg, db, coef))
    for a, b in zip(*res):
        assert torch.equal(a, b)
    # fp32 reference of the apply from the same coefficients
    a_, b_, c_ = res[1][3].view(3, C)
    xf = x.float()
    g = torch.where(xf * scale + shift > 0, dy.float(), torch.zeros_like(xf))
    ref = a_ * g - b_ - c_ * (xf - mean) * rstd + (0 if ad is None else ad.float())
    assert ((res[0][0].float() - ref).abs().max() / ref.abs().max()).item() < 1e-2
