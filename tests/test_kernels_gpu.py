"""Numerics of every HIP kernel against the plain-PyTorch fp32 reference of the
same op (ops/reference.py).  Shapes are the SURVEY Appendix-A shape classes
(scaled-down batch), plus the awkward cases: stride-2 fixed padding, 1x1
stride-2 projections, the 7x7/2 stem, channel padding, partial tiles."""
import math

import pytest
import torch

from distributed_tensorflow_resnet_amd.ops import functional as fn
from distributed_tensorflow_resnet_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


def _rel(a, b):
    a = a.float().cpu()
    b = b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _bf(t):
    return t.to(BF).float()


CONV_CASES = [
    # N, H, C, K, k, s
    (4, 32, 16, 16, 3, 1),
    (4, 32, 16, 16, 1, 1),
    (4, 32, 16, 32, 3, 2),
    (4, 32, 16, 32, 1, 2),
    (4, 16, 32, 32, 3, 1),
    (4, 16, 32, 64, 3, 2),
    (4, 8, 64, 64, 3, 1),
    (2, 14, 256, 1024, 1, 1),
    (2, 14, 256, 256, 3, 1),
    (2, 28, 128, 128, 3, 2),
    (2, 28, 512, 1024, 1, 2),
    (2, 7, 512, 2048, 1, 1),
    (3, 9, 32, 48, 3, 2),      # odd sizes / partial tiles
]


@pytest.mark.parametrize("N,H,C,K,k,s", CONV_CASES)
def test_conv_fwd(gpu, N, H, C, K, k, s):
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C, device=gpu).to(BF)
    w = (torch.randn(k, k, C, K, device=gpu) / math.sqrt(k * k * C)).to(BF)
    y = fn.conv2d_fwd(x, w.permute(3, 0, 1, 2).contiguous(), s)
    r = ref.conv2d(x.float(), w.float(), s)
    assert y.shape == r.shape
    assert _rel(y, r) < 1e-2


@pytest.mark.parametrize("N,H,C,K,k,s", CONV_CASES)
def test_conv_dgrad(gpu, N, H, C, K, k, s):
    torch.manual_seed(1)
    x = torch.randn(N, H, H, C, device=gpu)
    w = (torch.randn(k, k, C, K, device=gpu) / math.sqrt(k * k * C)).to(BF)
    x.requires_grad_(True)
    r = ref.conv2d(x, w.float(), s)
    dy = torch.randn_like(r).to(BF)
    r.backward(dy.float())
    dx = fn.conv2d_dgrad(dy, w.contiguous(), tuple(x.shape), s)
    assert _rel(dx, x.grad) < 1e-2


@pytest.mark.parametrize("N,H,C,K,k,s", CONV_CASES)
def test_conv_wgrad(gpu, N, H, C, K, k, s):
    torch.manual_seed(2)
    x = torch.randn(N, H, H, C, device=gpu).to(BF)
    w = torch.zeros(k, k, C, K, device=gpu, requires_grad=True)
    r = ref.conv2d(x.float(), w, s)
    dy = torch.randn_like(r).to(BF)
    r.backward(dy.float())
    dw = fn.conv2d_wgrad(dy, x, k, k, s)
    assert dw.shape == w.shape
    assert _rel(dw, w.grad) < 1e-2


def test_conv_stem_padded_channels(gpu):
    """CIFAR stem: 3 real channels zero-padded to 8; wgrad drops the pad."""
    torch.manual_seed(3)
    x3 = torch.randn(4, 32, 32, 3, device=gpu)
    x8 = torch.zeros(4, 32, 32, 8, device=gpu)
    x8[..., :3] = x3
    w = torch.randn(3, 3, 3, 16, device=gpu) * 0.2
    w8 = torch.zeros(16, 3, 3, 8, device=gpu)
    w8[..., :3] = w.permute(3, 0, 1, 2)
    y = fn.conv2d_fwd(x8.to(BF), w8.to(BF), 1)
    r = ref.conv2d(_bf(x3), _bf(w), 1)
    assert _rel(y, r) < 1e-2
    dy = torch.randn_like(r).to(BF)
    wt = torch.zeros_like(w, requires_grad=True)
    ref.conv2d(_bf(x3), wt, 1).backward(dy.float())
    g = torch.empty(3, 3, 3, 16, device=gpu)
    nat = fn.native()
    geom = fn.ConvGeom(4, 32, 32, 8, 16, 3, 3, 1)
    sp, pps = nat.wgrad_pick_splits(geom.as_list())
    part = torch.empty(sp * 16 * 9 * 8, device=gpu)
    st = fn._stream()
    nat.conv_wgrad(dy.data_ptr(), x8.to(BF).data_ptr(), 0, 0, part.data_ptr(), geom.as_list(), sp,
                   pps, st)
    nat.wgrad_reduce(part.data_ptr(), g.data_ptr(), sp, 16, 16, 9, 8, 3, 1.0, 0, st)
    assert _rel(g, wt.grad) < 1e-2


def test_conv_imagenet_stem(gpu):
    torch.manual_seed(4)
    x3 = torch.randn(2, 64, 64, 3, device=gpu)
    x8 = torch.zeros(2, 64, 64, 8, device=gpu)
    x8[..., :3] = x3
    w = torch.randn(7, 7, 3, 64, device=gpu) * 0.1
    w8 = torch.zeros(64, 7, 7, 8, device=gpu)
    w8[..., :3] = w.permute(3, 0, 1, 2)
    y = fn.conv2d_fwd(x8.to(BF), w8.to(BF), 2)
    r = ref.conv2d(_bf(x3), _bf(w), 2)
    assert y.shape == (2, 32, 32, 64)
    assert _rel(y, r) < 1e-2


def test_conv_fused_prologue_epilogue(gpu):
    """PRE (BN+ReLU on load, zero padding stays zero), residual add, BN stats."""
    torch.manual_seed(5)
    N, H, C, K = 4, 16, 32, 32
    x = torch.randn(N, H, H, C, device=gpu).to(BF)
    sc = torch.rand(C, device=gpu) + 0.5
    sh = torch.randn(C, device=gpu) * 0.3
    w = (torch.randn(3, 3, C, K, device=gpu) / math.sqrt(9 * C)).to(BF)
    res = torch.randn(N, H, H, K, device=gpu).to(BF)
    tiles, rows = fn.stat_tiles(N * H * H, K)
    part = torch.empty(tiles * 2 * K, device=gpu)
    y = fn.conv2d_fwd(x, w.permute(3, 0, 1, 2).contiguous(), 1, pre_scale=sc, pre_shift=sh,
                      residual=res, stat_part=part)
    a = torch.relu(x.float() * sc + sh).to(BF).float()
    r = ref.conv2d(a, w.float(), 1) + res.float()
    assert _rel(y, r) < 1e-2
    # stats of the bf16 output through bn_finalize
    gamma = torch.rand(K, device=gpu) + 0.5
    beta = torch.randn(K, device=gpu)
    mm = torch.zeros(K, device=gpu)
    mv = torch.ones(K, device=gpu)
    mean, rstd, scale, shift = fn.bn_finalize(part, tiles, rows, N * H * H, gamma, beta, mm, mv)
    yf = y.float().reshape(-1, K)
    _, m_ref, v_ref, uv_ref = ref.batch_norm_train(yf, gamma, beta)
    torch.testing.assert_close(mean, m_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rstd, torch.rsqrt(v_ref + 1.001e-5), rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(mm, 0.003 * m_ref, rtol=1e-3, atol=1e-6)
    torch.testing.assert_close(mv, 0.997 + 0.003 * uv_ref, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(scale, gamma * rstd)
    torch.testing.assert_close(shift, beta - mean * gamma * rstd)


@pytest.mark.parametrize("M,C,with_add", [(3000, 64, True), (1000, 2048, False),
                                          (70000, 256, True), (4097, 16, False)])
def test_bn_stats_and_backward(gpu, M, C, with_add):
    """BN stats/finalize/backward; the larger cases run several grid-stride rounds
    of the apply kernel (4096-block cap) and every channel-group width."""
    torch.manual_seed(6)
    x = (torch.randn(M, C, device=gpu) * 2 + 3).to(BF)
    part, tiles, rows = fn.bn_stats(x)
    gamma = torch.rand(C, device=gpu) + 0.5
    beta = torch.randn(C, device=gpu) * 0.1
    mm, mv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    mean, rstd, scale, shift = fn.bn_finalize(part, tiles, rows, M, gamma, beta, mm, mv)
    xf = x.float().requires_grad_(True)
    g_ = gamma.clone().requires_grad_(True)
    b_ = beta.clone().requires_grad_(True)
    y, m_ref, v_ref, _ = ref.batch_norm_train(xf, g_, b_)
    torch.testing.assert_close(mean, m_ref.detach(), rtol=1e-4, atol=1e-4)
    a = torch.relu(y)
    dy = torch.randn(M, C, device=gpu).to(BF)
    add = torch.randn(M, C, device=gpu).to(BF) if with_add else None
    a.backward(dy.float())
    dx, dgamma, dbeta = fn.bn_relu_backward(dy, x, mean, rstd, scale, shift, gamma, add=add)
    base = add.float() if with_add else 0.0
    assert _rel(dx.float() - base, xf.grad) < 2e-2
    assert _rel(dgamma, g_.grad) < 1e-3
    assert _rel(dbeta, b_.grad) < 1e-3
    y2 = fn.bn_relu_apply(x, scale, shift)
    assert _rel(y2, a) < 1e-2


def test_head_pool_xent(gpu):
    torch.manual_seed(7)
    N, HW, C, classes = 64, 8, 64, 10
    x = torch.randn(N, HW, HW, C, device=gpu).to(BF)
    sc = torch.rand(C, device=gpu) + 0.5
    sh = torch.randn(C, device=gpu) * 0.2
    pooled = fn.bnrelu_avgpool(x, sc, sh)
    r = torch.relu(x.float() * sc + sh).mean(dim=(1, 2))
    assert _rel(pooled, r) < 1e-2
    ld = 16
    logits = torch.zeros(N, ld, device=gpu)
    logits[:, :classes] = torch.randn(N, classes, device=gpu) * 3
    labels = torch.randint(0, classes, (N,), device=gpu)
    loss, corr, dl, db, probs = fn.softmax_xent(logits, labels, classes, 1.0 / N, want_probs=True)
    z = logits[:, :classes].clone().requires_grad_(True)
    lr_ = ref.softmax_cross_entropy(z, labels)
    lr_.backward()
    assert abs(loss.item() / N - lr_.item()) < 1e-4
    acc = (z.argmax(1) == labels).float().sum().item()
    assert corr.item() == acc
    assert _rel(dl[:, :classes], z.grad) < 1e-2
    assert torch.all(dl[:, classes:] == 0)
    torch.testing.assert_close(db, z.grad.sum(0), rtol=1e-4, atol=1e-6)
    dp = torch.randn(N, C, device=gpu).to(BF)
    dx = fn.avgpool_bwd(dp, HW, HW)
    torch.testing.assert_close(dx.float(), (dp.float() / (HW * HW))[:, None, None, :].expand(N, HW, HW, C),
                               rtol=1e-2, atol=1e-3)


@pytest.mark.parametrize("H,k,stride", [(112, 3, 2), (113, 3, 2), (15, 3, 2), (56, 3, 1), (28, 2, 2)])
def test_maxpool(gpu, H, k, stride):
    """TF SAME max pool vs the padded PyTorch pool: the stem's 3x3 / 2, odd sizes (a top /
    left pad of 1), stride 1 and a 2x2 window."""
    torch.manual_seed(8)
    x = torch.randn(2, H, H, 64, device=gpu).to(BF)
    y, am = fn.maxpool_fwd(x, k, stride)
    xf = x.float().requires_grad_(True)
    r = ref.max_pool_same(xf, k, stride)
    Ho = -(-H // stride)
    assert y.shape == r.shape == (2, Ho, Ho, 64)
    torch.testing.assert_close(y.float(), r.detach())
    dy = torch.randn_like(r).to(BF)
    r.backward(dy.float())
    dx = fn.maxpool_bwd(am, dy, tuple(x.shape), k, stride)
    assert _rel(dx, xf.grad) < 1e-2


def test_cifar_augment(gpu):
    torch.manual_seed(9)
    img = torch.randint(0, 256, (8, 3, 32, 32), dtype=torch.uint8, device=gpu)
    out, log = fn.cifar_augment(img, cpad=8, pad=4, seed=123, train=True, log_crops=True)
    assert out.shape == (8, 32, 32, 8)
    for n in range(8):
        oy, ox, flip = log[n].tolist()
        hwc = img[n].permute(1, 2, 0).float()
        padded = torch.zeros(40, 40, 3, device=gpu)
        padded[4:36, 4:36] = hwc
        crop = padded[oy:oy + 32, ox:ox + 32]
        if flip:
            crop = crop.flip(1)
        r = ref.per_image_standardization(crop)
        assert _rel(out[n, :, :, :3], r) < 1e-2
        assert torch.all(out[n, :, :, 3:] == 0)
    ev = fn.cifar_augment(img, cpad=8, train=False)
    r0 = ref.per_image_standardization(img[0].permute(1, 2, 0))
    assert _rel(ev[0, :, :, :3], r0) < 1e-2


@pytest.mark.parametrize("N,H,C,K,k,s", [(4, 16, 32, 64, 3, 1), (2, 28, 128, 512, 1, 1),
                                         (4, 32, 16, 32, 3, 2)])
def test_dgrad_fused_bn_backward_partials(gpu, N, H, C, K, k, s):
    """dgrad epilogue BNB: per-tile (sum g, sum g*xhat) == standalone reduction."""
    torch.manual_seed(10)
    x = torch.randn(N, H, H, C, device=gpu).to(BF)           # BN input (pre-activation)
    w = (torch.randn(k, k, C, K, device=gpu) / math.sqrt(k * k * C)).to(BF)
    g = fn.ConvGeom(N, H, H, C, K, k, k, s)
    dy = torch.randn(N, g.Ho, g.Wo, K, device=gpu).to(BF)
    mean = torch.randn(C, device=gpu) * 0.1
    rstd = torch.rand(C, device=gpu) + 0.5
    scale = torch.rand(C, device=gpu) + 0.5
    shift = torch.randn(C, device=gpu) * 0.2
    M = N * H * H
    tiles = -(-M // fn.native().conv_gemm_bm(M, C))
    part = torch.zeros(tiles * 2 * C, device=gpu)
    dx = fn.conv2d_dgrad(dy, w.contiguous(), tuple(x.shape), s,
                         bnb=(x, mean, rstd, scale, shift, part))
    dx_ref = fn.conv2d_dgrad(dy, w.contiguous(), tuple(x.shape), s)
    torch.testing.assert_close(dx.float(), dx_ref.float(), rtol=0, atol=0)
    xf = x.float().reshape(-1, C)
    gg = dx.float().reshape(-1, C) * ((xf * scale + shift) > 0).float()
    sg = gg.sum(0)
    sgx = (gg * (xf - mean) * rstd).sum(0)
    p = part.view(tiles, 2, C).sum(0)
    torch.testing.assert_close(p[0], sg, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(p[1], sgx, rtol=1e-4, atol=1e-3)


@pytest.fixture
def generic_conv():
    """Run a block with the direct 3x3 kernel disabled, then re-enable it."""
    nat = fn.native()

    class _Ctx:
        def __enter__(self):
            nat.set_conv_direct(0)

        def __exit__(self, *a):
            nat.set_conv_direct(1)
    return _Ctx()


# Every instantiation of the direct 3x3/s1 kernel (conv_direct.hip): (C, W, BM)
# = (16, 32, 256|64), (32, 16, 128|64), (64, 8, 64); BM follows conv_gemm_bm.
@pytest.mark.parametrize("N,H,C", [(128, 32, 16), (8, 32, 16), (256, 16, 32), (8, 16, 32),
                                   (16, 8, 64)])
def test_direct_conv3x3_matches_reference_and_generic(gpu, generic_conv, N, H, C):
    torch.manual_seed(11)
    M = N * H * H
    x = torch.randn(N, H, H, C, device=gpu).to(BF)
    w = (torch.randn(3, 3, C, C, device=gpu) / math.sqrt(9 * C)).to(BF)
    w_ohwi = w.permute(3, 0, 1, 2).contiguous()
    sc = torch.rand(C, device=gpu) + 0.5
    sh = torch.randn(C, device=gpu) * 0.3
    res = torch.randn(N, H, H, C, device=gpu).to(BF)
    tiles, rows = fn.stat_tiles(M, C)
    outs = []
    for direct in (True, False):
        part = torch.zeros(tiles * 2 * C, device=gpu)
        bpart = torch.zeros(tiles * 2 * C, device=gpu)
        mean = torch.randn(C, device=gpu) * 0.1
        rstd = torch.rand(C, device=gpu) + 0.5
        if direct:
            y = fn.conv2d_fwd(x, w_ohwi, 1, pre_scale=sc, pre_shift=sh, residual=res,
                              stat_part=part)
            dx = fn.conv2d_dgrad(res, w, tuple(x.shape), 1, bnb=(x, mean * 0, rstd * 0 + 1, sc,
                                                                   sh, bpart))
        else:
            with generic_conv:
                y = fn.conv2d_fwd(x, w_ohwi, 1, pre_scale=sc, pre_shift=sh, residual=res,
                                  stat_part=part)
                dx = fn.conv2d_dgrad(res, w, tuple(x.shape), 1,
                                     bnb=(x, mean * 0, rstd * 0 + 1, sc, sh, bpart))
        outs.append((y, part.view(tiles, 2, C), dx, bpart.view(tiles, 2, C)))
    a = torch.relu(x.float() * sc + sh).to(BF).float()
    r = ref.conv2d(a, w.float(), 1) + res.float()
    assert _rel(outs[0][0], r) < 1e-2
    assert _rel(outs[0][0], outs[1][0]) < 1e-2
    torch.testing.assert_close(outs[0][1][:, 0], outs[1][1][:, 0], rtol=2e-2, atol=2e-2)
    # dgrad: dx = conv_transpose(res, w); reference via autograd of the fp32 conv
    xr = torch.zeros(N, H, H, C, device=gpu, requires_grad=True)
    ref.conv2d(xr, w.float(), 1).backward(res.float())
    assert _rel(outs[0][2], xr.grad) < 1e-2
    assert _rel(outs[0][2], outs[1][2]) < 1e-2
    sums_d, sums_g = outs[0][3].sum(0), outs[1][3].sum(0)
    assert _rel(sums_d, sums_g) < 2e-2


@pytest.mark.parametrize("N,H,C,group", [(8, 32, 16, 0), (128, 32, 16, 16), (64, 16, 32, 16),
                                         (4, 14, 256, 0), (16, 14, 256, 16)])
def test_fused_last_arriver_bn_finalize(gpu, N, H, C, group):
    """In-kernel BN finalize (one- and two-level last arriver) == separate kernels,
    run twice to check the counters are left zeroed for the next launch."""
    torch.manual_seed(12)
    nat = fn.native()
    M = N * H * H
    x = torch.randn(N, H, H, C, device=gpu).to(BF)
    w = (torch.randn(3, 3, C, C, device=gpu) / math.sqrt(9 * C)).to(BF)
    w_ohwi = w.permute(3, 0, 1, 2).contiguous()
    tiles, rows = fn.stat_tiles(M, C)
    gamma = torch.rand(C, device=gpu) + 0.5
    beta = torch.randn(C, device=gpu)
    cnt = torch.zeros(4096, dtype=torch.int32, device=gpu)
    gpart = torch.empty(128 * 2 * C, device=gpu)
    for _ in range(2):
        part = torch.empty(tiles * 2 * C, device=gpu)
        mm, mv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
        mean, rstd, scale, shift = (torch.empty(C, device=gpu) for _ in range(4))
        y = fn.conv2d_fwd(x, w_ohwi, 1, stat_part=part,
                          fin=[cnt, gamma, beta, mm, mv, mean, rstd, scale, shift, gpart, group,
                              0])
        mm2, mv2 = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
        r = fn.bn_finalize(part, tiles, rows, M, gamma, beta, mm2, mv2)
        torch.testing.assert_close(mean, r[0], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(rstd, r[1], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(scale, r[2], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(shift, r[3], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(mm, mm2, rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(mv, mv2, rtol=1e-5, atol=1e-7)
        assert int(cnt.abs().sum()) == 0
        # backward: dgrad + BN-backward sums finalized in-kernel
        dy = torch.randn_like(y)
        bpart = torch.empty(tiles * 2 * C, device=gpu)
        dg, db, coef = torch.empty(C, device=gpu), torch.empty(C, device=gpu), \
            torch.empty(3 * C, device=gpu)
        fn.conv2d_dgrad(dy, w, tuple(x.shape), 1, bnb=(x, mean, rstd, scale, shift, bpart),
                        bfin=[cnt, gamma, rstd, dg, db, coef, gpart, group, 0])
        p = bpart.view(tiles, 2, C).sum(0)
        torch.testing.assert_close(db, p[0], rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(dg, p[1], rtol=1e-4, atol=1e-3)
        a = gamma * rstd
        torch.testing.assert_close(coef, torch.cat([a, a * db / M, a * dg / M]), rtol=1e-5,
                                   atol=1e-6)
        assert int(cnt.abs().sum()) == 0
    assert nat.conv_gemm_bn(M, C) in (16, 32, 64, 128)


@pytest.mark.parametrize("N,H,C,k,groups", [(8, 32, 16, 3, False), (128, 32, 16, 3, True),
                                            (64, 16, 32, 3, True), (16, 8, 64, 3, False),
                                            (4, 14, 128, 1, False), (8, 14, 128, 1, True),
                                            (128, 32, 16, 3, False), (128, 16, 32, 3, False),
                                            (128, 8, 64, 3, False)])
def test_consumer_prologue_bn_finalize(gpu, N, H, C, k, groups):
    """BnPreFin: the first consumer conv combines the producer's (mean, M2) partials
    (tile partials, or group partials left by groups_only last arrivers) in its
    prologue == bn_finalize + plain PRE; block 0 writes the BN outputs."""
    torch.manual_seed(13)
    nat = fn.native()
    M = N * H * H
    x = torch.randn(N, H, H, C, device=gpu).to(BF)
    w0 = (torch.randn(C, k, k, C, device=gpu) / math.sqrt(k * k * C)).to(BF)
    w1 = (torch.randn(C, k, k, C, device=gpu) / math.sqrt(k * k * C)).to(BF)
    bm = nat.conv_gemm_bm(M, C)
    T = -(-M // bm)
    part = torch.empty(T * 2 * C, device=gpu)
    gamma = torch.rand(C, device=gpu) + 0.5
    beta = torch.randn(C, device=gpu)
    fin = None
    src, cnt, rows = part, T, bm
    if not groups:
        assert T <= nat.pfin_cap(C)
    if groups:
        cap = (256 // C) * 8
        gs = 2
        while -(-T // gs) > cap:
            gs *= 2
        gpart = torch.empty(-(-T // gs) * 2 * C, device=gpu)
        cntr = torch.zeros(4096, dtype=torch.int32, device=gpu)
        fin = [cntr, gamma, beta, 0, 0, 0, 0, 0, 0, gpart, gs, 1]
        src, cnt, rows = gpart, -(-T // gs), gs * bm
    y0 = fn.conv2d_fwd(x, w0, 1, stat_part=part, fin=fin)
    if groups:
        assert int(cntr.abs().sum()) == 0
    outs = [torch.empty(C, device=gpu) for _ in range(4)]
    mm, mv = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    y1 = fn.conv2d_fwd(y0, w1, 1, pre_scale=outs[2], pre_shift=outs[3],
                       pfin=[src, cnt, rows, M, gamma, beta, *outs, mm, mv])
    mm2, mv2 = torch.zeros(C, device=gpu), torch.ones(C, device=gpu)
    r = fn.bn_finalize(part, T, bm, M, gamma, beta, mm2, mv2)
    for a, b in zip(outs, r):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(mm, mm2, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(mv, mv2, rtol=1e-5, atol=1e-7)
    y1_ref = fn.conv2d_fwd(y0, w1, 1, pre_scale=r[2], pre_shift=r[3])
    assert _rel(y1, y1_ref) < 2e-3


@pytest.mark.parametrize("N,H,C", [(8, 32, 16), (4, 16, 32), (6, 8, 64), (128, 32, 16),
                                   # batch-adaptive tiles (pixels, taps per workgroup):
                                   (16, 32, 16), (16, 16, 32), (8, 16, 32), (2, 16, 32),
                                   (16, 8, 64), (32, 8, 64), (64, 8, 64)])
def test_direct_wgrad_matches_reference_and_generic(gpu, N, H, C):
    """Halo-tiled 3x3/s1 wgrad (conv_wgrad_direct.hip) with the fused BN+ReLU of x:
    == fp32 autograd of conv(relu(x*scale+shift)) and == the generic split-K kernel."""
    torch.manual_seed(14)
    nat = fn.native()
    x = torch.randn(N, H, H, C, device=gpu).to(BF)
    sc = torch.rand(C, device=gpu) + 0.5
    sh = torch.randn(C, device=gpu) * 0.3
    dy = torch.randn(N, H, H, C, device=gpu).to(BF)
    pps = nat.wgrad_pick_splits([N, H, H, C, H, H, C, 3, 3, 1, 1])[1]
    # (the selection gives <= 1024-pixel 64-channel wgrads to the split-K kernel)
    if not (C == 64 and N * H * H <= 1024):
        assert pps in (64, 128, 256, 512, 1024)
    dw = fn.conv2d_wgrad(dy, x, 3, 3, 1, pre_scale=sc, pre_shift=sh)
    nat.set_wgrad_direct(0)
    try:
        dw_gen = fn.conv2d_wgrad(dy, x, 3, 3, 1, pre_scale=sc, pre_shift=sh)
    finally:
        nat.set_wgrad_direct(1)
    a = torch.relu(x.float() * sc + sh).to(BF).float()
    w = torch.zeros(3, 3, C, C, device=gpu, requires_grad=True)
    ref.conv2d(a, w, 1).backward(dy.float())
    assert _rel(dw, w.grad) < 1e-3
    assert _rel(dw, dw_gen) < 1e-3


@pytest.mark.parametrize("N,H,C,with_add,cnt", [(8, 32, 16, True, 16), (128, 32, 16, False, 16),
                                                (16, 16, 32, True, 16), (16, 8, 64, False, 16),
                                                (128, 32, 16, True, 512), (128, 16, 32, False, 512),
                                                (128, 8, 64, True, 128)])
def test_direct_dgrad_fused_bn_backward(gpu, N, H, C, with_add, cnt):
    """BnBwdPre: the direct dgrad applies the pending BN+ReLU backward to its input
    while staging (dh = a*g - b - c*xhat + add, coefficients combined from the
    producer's partial sums), writes dh, and == bn_bwd_finalize + bn_bwd_apply + dgrad."""
    torch.manual_seed(15)
    nat = fn.native()
    M = N * H * H
    da = torch.randn(N, H, H, C, device=gpu).to(BF)          # grad wrt relu(bn(x))
    x = torch.randn(N, H, H, C, device=gpu).to(BF)           # BN input
    add = torch.randn(N, H, H, C, device=gpu).to(BF) if with_add else None
    w = (torch.randn(3, 3, C, C, device=gpu) / math.sqrt(9 * C)).to(BF)
    mean = torch.randn(C, device=gpu) * 0.1
    rstd = torch.rand(C, device=gpu) + 0.5
    gamma = torch.rand(C, device=gpu) + 0.5
    scale = gamma * rstd
    shift = torch.randn(C, device=gpu) * 0.2 - mean * scale
    # partial sums (sum g, sum g*xhat) in 16 row blocks, as a producer epilogue would
    xf, gf = x.float().reshape(-1, C), da.float().reshape(-1, C)
    g = gf * ((xf * scale + shift) > 0).float()
    xh = (xf - mean) * rstd
    assert cnt <= nat.pfin_cap(C)
    part = torch.stack([torch.stack([gg.sum(0), (gg * hh).sum(0)])
                        for gg, hh in zip(g.chunk(cnt), xh.chunk(cnt))]).contiguous()
    dh = torch.empty_like(da)
    dg, db, coef = (torch.empty(n, device=gpu) for n in (C, C, 3 * C))
    dx = fn.conv2d_dgrad(da, w, tuple(x.shape), 1,
                         abwd=[x, 0 if add is None else add, mean, rstd, scale, shift, gamma,
                               part, cnt, dh, dg, db, coef])
    assert nat.conv_direct_covers(1, [N, H, H, C, H, H, C, 3, 3, 1, 1])
    # reference: separate finalize + apply, then the plain dgrad of the applied tensor
    dg2, db2, coef2 = (torch.empty(n, device=gpu) for n in (C, C, 3 * C))
    nat.bn_bwd_finalize(part.data_ptr(), cnt, M, C, gamma.data_ptr(), rstd.data_ptr(),
                        dg2.data_ptr(), db2.data_ptr(), coef2.data_ptr(),
                        torch.cuda.current_stream().cuda_stream)
    dh2 = torch.empty_like(da)
    nat.bn_bwd_apply(da.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                     scale.data_ptr(), shift.data_ptr(), coef2.data_ptr(),
                     0 if add is None else add.data_ptr(), dh2.data_ptr(), M, C,
                     torch.cuda.current_stream().cuda_stream)
    torch.testing.assert_close(dg, dg2, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(db, db2, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(coef, coef2, rtol=1e-5, atol=1e-6)
    assert (dh.float() - dh2.float()).abs().max().item() <= 2 * 2 ** -8 * dh2.float().abs().max().item()
    dx2 = fn.conv2d_dgrad(dh2, w, tuple(x.shape), 1)
    assert _rel(dx, dx2) < 5e-3


def test_direct_dgrad_fused_bn_backward_precomputed_coef(gpu):
    """BnBwdPre with cnt = 0: coefficients read from a prior bn_bwd_finalize."""
    torch.manual_seed(16)
    nat = fn.native()
    N, H, C = 16, 16, 32
    M = N * H * H
    da = torch.randn(N, H, H, C, device=gpu).to(BF)
    x = torch.randn(N, H, H, C, device=gpu).to(BF)
    add = torch.randn(N, H, H, C, device=gpu).to(BF)
    w = (torch.randn(3, 3, C, C, device=gpu) / math.sqrt(9 * C)).to(BF)
    mean, rstd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    gamma = torch.rand(C, device=gpu) + 0.5
    scale, shift = gamma * rstd, torch.randn(C, device=gpu) * 0.2
    part = torch.randn(4, 2, C, device=gpu).contiguous()
    dg, db, coef = (torch.empty(n, device=gpu) for n in (C, C, 3 * C))
    st = torch.cuda.current_stream().cuda_stream
    nat.bn_bwd_finalize(part.data_ptr(), 4, M, C, gamma.data_ptr(), rstd.data_ptr(),
                        dg.data_ptr(), db.data_ptr(), coef.data_ptr(), st)
    dh = torch.empty_like(da)
    dx = fn.conv2d_dgrad(da, w, tuple(x.shape), 1,
                         abwd=[x, add, mean, rstd, scale, shift, gamma, 0, 0, dh, dg, db, coef])
    dh2 = torch.empty_like(da)
    nat.bn_bwd_apply(da.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                     scale.data_ptr(), shift.data_ptr(), coef.data_ptr(), add.data_ptr(),
                     dh2.data_ptr(), M, C, st)
    torch.testing.assert_close(dh.float(), dh2.float(), rtol=0, atol=0)
    assert _rel(dx, fn.conv2d_dgrad(dh2, w, tuple(x.shape), 1)) < 5e-3


def test_grouped_wgrad_reduce_wide_and_deep(gpu):
    """wgrad_reduce_grouped over convs of both work-unit shapes (few splits: the
    transposed 16x64 tile; many: the 256-column split-row form), with padded output
    (Kv < K) and input (Cv < C) channels dropped, == sum over splits in HWIO."""
    import numpy as np

    from distributed_tensorflow_resnet_amd.train.engine import WGD_DTYPE

    torch.manual_seed(17)
    nat = fn.native()
    cases = [(3, 512, 9, 512, 512, 512), (1, 64, 1, 256, 64, 256), (8, 32, 9, 24, 20, 24),
             (96, 64, 1, 256, 64, 256), (12, 16, 9, 8, 10, 3), (5, 1024, 1, 2048, 1001, 2048)]
    parts, grads, refs = [], [], []
    arr = np.zeros(len(cases), dtype=WGD_DTYPE)
    chunk = 0
    for i, (sp, K, taps, C, Kv, Cv) in enumerate(cases):
        p = torch.randn(sp, K, taps * C, device=gpu)
        g = torch.full((taps, Cv, Kv), 7.0, device=gpu)
        ref = p.double().sum(0).view(K, taps, C)[:Kv, :, :Cv].permute(1, 2, 0) * 0.5
        parts.append(p)
        grads.append(g)
        refs.append(ref)
        arr[i] = (p.data_ptr(), g.data_ptr(), sp, K, Kv, taps, C, Cv, chunk)
        chunk += nat.wgrad_reduce_chunks(sp, K, taps, C)
    t = torch.from_numpy(arr.view(np.uint8).copy()).to(gpu)
    nat.wgrad_reduce_grouped(t.data_ptr(), len(cases), chunk, 0.5, fn._stream())
    torch.cuda.synchronize()
    for (sp, K, taps, C, Kv, Cv), g, r in zip(cases, grads, refs):
        torch.testing.assert_close(g.double(), r, rtol=1e-5, atol=1e-5 * sp ** 0.5,
                                   msg=lambda m: f"{(sp, K, taps, C, Kv, Cv)}: {m}")


@pytest.mark.parametrize("N,H,C,K,k,pre", [(128, 7, 512, 512, 3, True), (128, 7, 2048, 512, 1, True),
                                           (64, 7, 512, 512, 3, False), (16, 14, 256, 256, 3, True)])
def test_splitk_conv_matches_unsplit(gpu, N, H, C, K, k, pre):
    """Split-K of the pipelined implicit GEMM (under-filled grids, the 7x7 stage): the
    slices' fp32 tiles summed by the last arriver == the one-slice result (to fp32
    summation order) and the fp32 reference; BN statistics likewise; repeated launches
    reuse the tickets (each last arriver resets its tile's)."""
    torch.manual_seed(18)
    nat = fn.native()
    x = torch.randn(N, H, H, C, device=gpu).to(BF)
    w = (torch.randn(K, k, k, C, device=gpu) / math.sqrt(k * k * C)).to(BF)
    sc = torch.rand(C, device=gpu) + 0.5
    sh = torch.randn(C, device=gpu) * 0.1
    kw = dict(pre_scale=sc, pre_shift=sh) if pre else {}
    M = N * H * H
    tiles, _ = fn.stat_tiles(M, K)
    outs, parts = [], []
    for slices in (1, 4, 2):
        nat.set_conv_splitk(slices)
        try:
            part = torch.zeros(tiles * 2 * K, device=gpu)
            for _ in range(3):
                out = fn.conv2d_fwd(x, w, 1, stat_part=part, **kw)
            torch.cuda.synchronize()
        finally:
            nat.set_conv_splitk(2)
        outs.append(out.float())
        parts.append(part.clone())
    a = torch.relu(x.float() * sc + sh) if pre else x.float()
    ref_out = ref.conv2d(a.to(BF).float(), w.float().permute(1, 2, 3, 0), 1)
    for o, p in zip(outs[1:], parts[1:]):
        assert _rel(o, outs[0]) < 2e-3
        torch.testing.assert_close(p, parts[0], rtol=1e-3, atol=1e-3)
    assert _rel(outs[2], ref_out) < 1e-2


@pytest.mark.parametrize("N,H,C,K,k", [(128, 7, 512, 512, 3), (128, 7, 512, 2048, 1)])
def test_splitk_dgrad_matches_unsplit(gpu, N, H, C, K, k):
    """The 7x7 dgrads run the pipelined loop split in two: == one slice and the
    fp32 reference, BN-backward sums (BNB epilogue) included."""
    torch.manual_seed(19)
    nat = fn.native()
    dy = torch.randn(N, H, H, K, device=gpu).to(BF)
    w = (torch.randn(k, k, C, K, device=gpu) / math.sqrt(k * k * K)).to(BF)
    x = torch.randn(N, H, H, C, device=gpu).to(BF)
    mean, rstd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    sc, sh = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu) * 0.1
    M = N * H * H
    outs, accs = [], []
    for slices in (1, 2):
        nat.set_conv_splitk(slices)
        try:
            acc = torch.zeros(8 * 2 * C, device=gpu, dtype=torch.float64)
            part = torch.zeros((M // 64 + 1) * 2 * C, device=gpu)
            out = fn.conv2d_dgrad(dy, w, tuple(x.shape), 1, bnb=(x, mean, rstd, sc, sh, part),
                                  bfin=[acc])
            torch.cuda.synchronize()
        finally:
            nat.set_conv_splitk(2)
        outs.append(out.float())
        accs.append(acc.view(8, 2, C).sum(0))
    wt = w.float().permute(0, 1, 2, 3)  # HWIO [kh][kw][C][K]
    xt = torch.zeros(N, H, H, C, device=gpu, requires_grad=True)
    ref.conv2d(xt, wt, 1).backward(dy.float())
    assert _rel(outs[1], outs[0]) < 2e-3
    assert _rel(outs[1], xt.grad) < 1e-2
    torch.testing.assert_close(accs[1], accs[0], rtol=2e-3, atol=1e-2)


@pytest.mark.parametrize("N,H,C,K,k,acc", [(64, 32, 16, 32, 3, False), (64, 32, 16, 32, 1, True),
                                           (32, 16, 32, 64, 3, False), (8, 56, 128, 128, 3, False),
                                           (8, 56, 256, 512, 1, True), (4, 14, 1024, 2048, 1, False),
                                           (8, 28, 256, 256, 3, True)])
def test_parity_class_stride2_dgrad(gpu, N, H, C, K, k, acc):
    """Stride-2 dgrad by output parity class (4 dense GEMMs over their own rows and
    taps, one launch) == the masked all-taps kernel and the fp32 reference, with the
    BN-backward sums (fp64 accumulators) and accumulate-into-output."""
    torch.manual_seed(20)
    nat = fn.native()
    g = fn.ConvGeom(N, H, H, C, K, k, k, 2)
    dy = torch.randn(N, g.Ho, g.Wo, K, device=gpu).to(BF)
    w = (torch.randn(k, k, C, K, device=gpu) / math.sqrt(k * k * K)).to(BF)
    x = torch.randn(N, H, H, C, device=gpu).to(BF)
    base = torch.randn(N, H, H, C, device=gpu).to(BF)
    mean, rstd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    sc, sh = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu) * 0.1
    M = N * H * H
    outs, accs = [], []
    for parity in (0, 1):
        nat.set_conv_parity(parity)
        try:
            bacc = torch.zeros(8 * 2 * C, device=gpu, dtype=torch.float64)
            part = torch.zeros((M // 64 + 1) * 2 * C, device=gpu)
            out = base.clone()
            fn.conv2d_dgrad(dy, w, tuple(x.shape), 2, out=out, accumulate=acc,
                            bnb=(x, mean, rstd, sc, sh, part), bfin=[bacc])
            torch.cuda.synchronize()
        finally:
            nat.set_conv_parity(1)
        outs.append(out.float())
        accs.append(bacc.view(8, 2, C).sum(0))
    xt = torch.zeros(N, H, H, C, device=gpu, requires_grad=True)
    ref.conv2d(xt, w.float(), 2).backward(dy.float())
    want = xt.grad + (base.float() if acc else 0)
    assert _rel(outs[1], outs[0]) < 1e-2
    assert _rel(outs[1], want) < 1e-2
    torch.testing.assert_close(accs[1], accs[0], rtol=1e-2, atol=1e-1)


RING_CASES = [
    # mode, N, H, C, K, k, s
    ("fwd", 32, 14, 256, 256, 3, 1),
    ("fwd", 32, 28, 128, 128, 3, 2),
    ("fwd", 32, 14, 512, 256, 1, 1),
    ("fwd", 128, 14, 512, 1024, 1, 2),
    ("fwd", 128, 7, 512, 512, 3, 1),      # split-K grid (196 tiles)
    ("dgrad", 32, 14, 256, 256, 3, 1),
    ("dgrad", 128, 14, 256, 256, 3, 2),   # stride 2: output-parity classes
    ("dgrad", 128, 7, 512, 2048, 1, 1),   # split-K, 1x1
    ("fwd", 48, 28, 64, 64, 3, 1),        # 128 x 64 tiles (64 output channels)
    ("fwd", 48, 28, 512, 64, 1, 1),
    ("dgrad", 48, 28, 64, 64, 3, 1),
    ("dgrad", 48, 28, 64, 256, 1, 1),
]


@pytest.mark.parametrize("mode,N,H,C,K,k,s", RING_CASES)
def test_ring_conv_matches_register_loop_and_reference(gpu, mode, N, H, C, K, k, s):
    """LDS-DMA ring loop (conv_ring.hip) == the register-staged loop (tune ring=0) to fp32
    summation order and == the fp32 reference, with the fused epilogues (forward:
    residual + BN statistics; dgrad: BN-backward sums into the fp64 accumulators +
    accumulate-into-output); padding taps read as zeros."""
    torch.manual_seed(21)
    nat = fn.native()
    dflt = {t[0]: t[1] for t in nat.tune_table()}
    g = fn.ConvGeom(N, H, H, C, K, k, k, s)
    fwd = mode == "fwd"
    assert nat.conv_ring_covers(0 if fwd else 1, g.as_list())
    if fwd:
        x = torch.randn(N, H, H, C, device=gpu).to(BF)
        w = (torch.randn(K, k, k, C, device=gpu) / math.sqrt(k * k * C)).to(BF)
        res = torch.randn(N, g.Ho, g.Wo, K, device=gpu).to(BF)
        tiles, _ = fn.stat_tiles(N * g.Ho * g.Wo, K)
    else:
        dy = torch.randn(N, g.Ho, g.Wo, K, device=gpu).to(BF)
        w = (torch.randn(k, k, C, K, device=gpu) / math.sqrt(k * k * K)).to(BF)
        x = torch.randn(N, H, H, C, device=gpu).to(BF)
        base = torch.randn(N, H, H, C, device=gpu).to(BF)
        mean, rstd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
        sc, sh = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu) * 0.1
    outs, sums = [], []
    for ring in (0, 1):
        nat.tune_set("ring", ring)
        try:
            for _ in range(2):   # repeated launches (split-K tickets are reset)
                if fwd:
                    part = torch.zeros(tiles * 2 * K, device=gpu)
                    out = fn.conv2d_fwd(x, w, s, residual=res, stat_part=part)
                    red = part
                else:
                    bacc = torch.zeros(8 * 2 * C, device=gpu, dtype=torch.float64)
                    part = torch.zeros((N * H * H // 64 + 1) * 2 * C, device=gpu)
                    out = base.clone()
                    fn.conv2d_dgrad(dy, w, tuple(x.shape), s, out=out, accumulate=True,
                                    bnb=(x, mean, rstd, sc, sh, part), bfin=[bacc])
                    red = bacc.view(8, 2, C).sum(0)
            torch.cuda.synchronize()
        finally:
            nat.tune_set("ring", dflt["ring"])
        outs.append(out.float())
        sums.append(red.float())
    if fwd:
        want = ref.conv2d(x.float(), w.float().permute(1, 2, 3, 0), s) + res.float()
    else:
        xt = torch.zeros(N, H, H, C, device=gpu, requires_grad=True)
        ref.conv2d(xt, w.float(), s).backward(dy.float())
        want = xt.grad + base.float()
    assert _rel(outs[1], outs[0]) < 2e-3
    assert _rel(outs[1], want) < 1e-2
    torch.testing.assert_close(sums[1], sums[0], rtol=2e-3, atol=2e-2)


@pytest.mark.parametrize("N,H,C,K,k,s", [(4, 28, 128, 128, 3, 1), (8, 14, 256, 256, 3, 2),
                                         (4, 56, 256, 128, 1, 1), (16, 7, 512, 512, 3, 1),
                                         (2, 14, 1024, 2048, 1, 2)])
def test_ring_wgrad_matches_register_loop_and_reference(gpu, N, H, C, K, k, s):
    """LDS-DMA ring weight gradient (conv_wgrad_ring.hip) with the BN+ReLU prologue
    applied in LDS (padding taps stay zero) == the register-staged loop (tune
    ring_wgrad=0) and the fp32 reference, over the split-K partial slabs + reduce."""
    torch.manual_seed(22)
    nat = fn.native()
    dflt = {t[0]: t[1] for t in nat.tune_table()}
    x = torch.randn(N, H, H, C, device=gpu).to(BF)
    g = fn.ConvGeom(N, H, H, C, K, k, k, s)
    dy = torch.randn(N, g.Ho, g.Wo, K, device=gpu).to(BF)
    sc, sh = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu) * 0.3
    outs = []
    for ring in (1, 0):
        nat.tune_set("ring_wgrad", ring)
        try:
            gw = torch.empty(k, k, C, K, device=gpu)
            fn.conv2d_wgrad(dy, x, k, k, s, grad_hwio=gw, pre_scale=sc, pre_shift=sh)
            torch.cuda.synchronize()
        finally:
            nat.tune_set("ring_wgrad", dflt["ring_wgrad"])
        outs.append(gw.clone())
    a = torch.relu(x.float() * sc + sh).to(BF).float()
    wt = torch.zeros(k, k, C, K, device=gpu, requires_grad=True)
    ref.conv2d(a, wt, s).backward(dy.float())
    assert _rel(outs[0], outs[1]) < 1e-4
    assert _rel(outs[0], wt.grad) < 1e-2


@pytest.mark.parametrize("N,H,C,K", [(8, 56, 256, 64), (8, 28, 512, 128), (2, 4, 256, 64),
                                     (4, 14, 1024, 128), (8, 14, 1024, 256), (4, 4, 256, 256),
                                     (16, 7, 2048, 512)])
def test_streaming_narrow_dgrad_bn_backward(gpu, N, H, C, K):
    """bnd1x1 (bn_dgrad1x1.hip): the sums pass == the implicit-GEMM dgrad's BN-backward
    sums (fp64 accumulators) to fp32 rounding, and the apply pass == bn_bwd_apply of the
    dgrad's stored gradient bitwise for the same coefficients (same MFMA order, same
    bf16 rounding of g, same apply arithmetic); dx == the fp32 reference."""
    torch.manual_seed(23)
    nat = fn.native()
    st = torch.cuda.current_stream().cuda_stream
    M = N * H * H
    assert nat.bnd1x1_covers(M, C, K)
    g = fn.ConvGeom(N, H, H, C, K, 1, 1, 1)
    dz = torch.randn(N, H, H, K, device=gpu).to(BF)
    w = (torch.randn(1, 1, C, K, device=gpu) / math.sqrt(K)).to(BF)
    x = torch.randn(N, H, H, C, device=gpu).to(BF)
    add = torch.randn(N, H, H, C, device=gpu).to(BF)
    mean = torch.randn(C, device=gpu) * 0.1
    rstd = torch.rand(C, device=gpu) + 0.5
    gamma = torch.rand(C, device=gpu) + 0.5
    sc, sh = gamma * rstd, torch.randn(C, device=gpu) * 0.2 - mean * gamma * rstd
    rep = nat.bn_acc_rep()
    # reference path: implicit-GEMM dgrad with BNB sums, finalize, separate apply
    bacc1 = torch.zeros(rep * 2 * C, device=gpu, dtype=torch.float64)
    part = torch.zeros((M // 16 + 1) * 2 * C, device=gpu)
    da = torch.empty(N, H, H, C, device=gpu, dtype=BF)
    nat.conv_gemm(1, dz.data_ptr(), w.data_ptr(), da.data_ptr(), 0, 0, 0, 0, 0, 0, 0, 0,
                  g.as_list(), [x.data_ptr(), mean.data_ptr(), rstd.data_ptr(), sc.data_ptr(),
                                sh.data_ptr(), part.data_ptr()], [], [bacc1.data_ptr()], [], [],
                  0.997, ref.BN_EPS, 1, st)
    coef1 = torch.empty(3 * C, device=gpu)
    dgb1 = torch.empty(2 * C, device=gpu)
    nat.bn_bwd_finalize(bacc1.data_ptr(), -1, M, C, gamma.data_ptr(), rstd.data_ptr(),
                        dgb1.data_ptr(), dgb1.data_ptr() + 4 * C, coef1.data_ptr(), st)
    want = torch.empty_like(da)
    nat.bn_bwd_apply(da.data_ptr(), x.data_ptr(), mean.data_ptr(), rstd.data_ptr(), sc.data_ptr(),
                     sh.data_ptr(), coef1.data_ptr(), add.data_ptr(), want.data_ptr(), M, C, st)
    # streaming kernel: sums, then apply with the reference coefficients
    bacc2 = torch.zeros_like(bacc1)
    base = [dz.data_ptr(), w.data_ptr(), x.data_ptr()]
    bnp = [mean.data_ptr(), rstd.data_ptr(), sc.data_ptr(), sh.data_ptr()]
    nat.bnd1x1(0, base + [0, 0] + bnp + [0, bacc2.data_ptr()], M, C, K, st)
    got = torch.full_like(da, float("nan"))
    nat.bnd1x1(1, base + [add.data_ptr(), got.data_ptr()] + bnp + [coef1.data_ptr(), 0], M, C, K,
               st)
    torch.cuda.synchronize()
    s1 = bacc1.view(rep, 2, C).sum(0)
    s2 = bacc2.view(rep, 2, C).sum(0)
    scale_ = s1.abs().max().item() + 1.0
    assert (s2 - s1).abs().max().item() <= 1e-5 * scale_
    torch.testing.assert_close(got.float(), want.float(), rtol=0, atol=0)
    dxt = torch.zeros(N, H, H, C, device=gpu, requires_grad=True)
    ref.conv2d(dxt, w.float(), 1).backward(dz.float())
    xf, gf = x.float().reshape(-1, C), dxt.grad.reshape(-1, C)
    gg = gf * ((xf * sc + sh) > 0).float()
    xh = (xf - mean) * rstd
    dx_ref = gamma * rstd * (gg - gg.mean(0) - xh * (gg * xh).mean(0)) + add.float().reshape(-1, C)
    assert _rel(got.reshape(-1, C), dx_ref) < 1e-2


@pytest.mark.parametrize("mode", ["pre", "pfin", "nopre"])
@pytest.mark.parametrize("N,H,K,C", [(8, 56, 64, 256), (8, 28, 128, 512), (8, 14, 256, 1024),
                                     (2, 4, 64, 256), (8, 56, 256, 64), (8, 28, 512, 128),
                                     (8, 14, 64, 64), (4, 14, 256, 128), (16, 7, 512, 2048)])
def test_streaming_narrow_fwd_bn_residual_stats(gpu, N, H, K, C, mode):
    """bnf1x1 (bn_fwd1x1.hip) == the implicit-GEMM forward with the same fusions (BN+ReLU
    prologue given or finalized from fp64 accumulators in the prologue, residual add, BN
    statistics into fp64 accumulators): output bitwise, statistics to fp64/fp32 rounding,
    the prologue's finalize outputs equal; and == the fp32 reference."""
    torch.manual_seed(24)
    nat = fn.native()
    st = torch.cuda.current_stream().cuda_stream
    M = N * H * H
    assert nat.bnf1x1_covers(M, C, K)
    rep = nat.bn_acc_rep()
    g = fn.ConvGeom(N, H, H, K, C, 1, 1, 1)
    x = torch.randn(N, H, H, K, device=gpu).to(BF)
    w = (torch.randn(C, 1, 1, K, device=gpu) / math.sqrt(K)).to(BF)   # OHWI
    res = torch.randn(N, H, H, C, device=gpu).to(BF)
    gamma, beta = torch.rand(K, device=gpu) + 0.5, torch.randn(K, device=gpu) * 0.1
    sc, sh = torch.rand(K, device=gpu) + 0.5, torch.randn(K, device=gpu) * 0.2
    # accumulator sums of a made-up producer of x: exactly x's own batch sums
    xf = x.float().reshape(-1, K).double()
    pacc = torch.zeros(rep, 2, K, device=gpu, dtype=torch.float64)
    pacc[0, 0], pacc[0, 1] = xf.sum(0), (xf * xf).sum(0)
    outs = []
    for kern in ("gemm", "stream"):
        out = torch.full((N, H, H, C), float("nan"), device=gpu, dtype=BF)
        sacc = torch.zeros(rep * 2 * C, device=gpu, dtype=torch.float64)
        bnout = [torch.zeros(K, device=gpu) for _ in range(4)] + [torch.zeros(K, device=gpu),
                                                                  torch.ones(K, device=gpu)]
        pf, ps, psh = [], 0, 0
        if mode == "pfin":
            pf = [pacc.data_ptr(), 0xFFFFFFFF, 0, M, gamma.data_ptr(), beta.data_ptr()] + \
                 [t.data_ptr() for t in bnout]
            ps, psh = bnout[2].data_ptr(), bnout[3].data_ptr()
        elif mode == "pre":
            ps, psh = sc.data_ptr(), sh.data_ptr()
        if kern == "gemm":
            nat.conv_gemm(0, x.data_ptr(), w.data_ptr(), out.data_ptr(), 0, res.data_ptr(), ps, psh,
                          0, 0, torch.zeros(1, device=gpu).data_ptr(), 0, g.as_list(), [],
                          [sacc.data_ptr()], [], pf, [], 0.997, ref.BN_EPS, 1, st)
        else:
            nat.bnf1x1([x.data_ptr(), w.data_ptr(), res.data_ptr(), out.data_ptr(),
                        0 if mode == "pfin" else ps, 0 if mode == "pfin" else psh,
                        sacc.data_ptr()], pf, M, C, K, 0.997, ref.BN_EPS, 1, st)
        torch.cuda.synchronize()
        outs.append((out, sacc.view(rep, 2, C).sum(0), [t.clone() for t in bnout]))
    (o0, s0, b0), (o1, s1, b1) = outs
    torch.testing.assert_close(o1.float(), o0.float(), rtol=0, atol=0)
    torch.testing.assert_close(s1, s0, rtol=1e-5, atol=1e-2)
    if mode == "pfin":
        for t0, t1 in zip(b0, b1):
            torch.testing.assert_close(t1, t0, rtol=1e-6, atol=1e-7)
        scale, shift = b1[2], b1[3]
    else:
        scale, shift = (sc, sh) if mode == "pre" else (None, None)
    a_in = x.float() if scale is None else torch.relu(x.float() * scale + shift).to(BF).float()
    want = ref.conv2d(a_in, w.float().permute(1, 2, 3, 0), 1) + res.float()
    assert _rel(o1, want) < 1e-2
    yf = o1.float().reshape(-1, C).double()
    torch.testing.assert_close(s1[0], yf.sum(0), rtol=1e-9, atol=1e-6)
    torch.testing.assert_close(s1[1], (yf * yf).sum(0), rtol=1e-9, atol=1e-6)


@pytest.mark.parametrize("N,H,C,K", [(8, 56, 64, 256), (8, 28, 128, 512), (8, 14, 1024, 256),
                                     (8, 14, 64, 64), (4, 14, 128, 256), (8, 28, 256, 64),
                                     (16, 7, 2048, 512)])
def test_streaming_dgrad_store_and_bn_backward_sums(gpu, N, H, C, K):
    """bnd1x1 mode 2 == the implicit-GEMM dgrad with the BNB epilogue: the stored dgrad
    bitwise (same MFMA order), the BN-backward sums to fp32 rounding, both vs the fp32
    reference."""
    torch.manual_seed(25)
    nat = fn.native()
    st = torch.cuda.current_stream().cuda_stream
    M = N * H * H
    assert nat.bnd1x1_covers(M, C, K)
    rep = nat.bn_acc_rep()
    g = fn.ConvGeom(N, H, H, C, K, 1, 1, 1)
    dz = torch.randn(N, H, H, K, device=gpu).to(BF)
    w = (torch.randn(1, 1, C, K, device=gpu) / math.sqrt(K)).to(BF)
    x = torch.randn(N, H, H, C, device=gpu).to(BF)
    mean, rstd = torch.randn(C, device=gpu) * 0.1, torch.rand(C, device=gpu) + 0.5
    sc, sh = torch.rand(C, device=gpu) + 0.5, torch.randn(C, device=gpu) * 0.2
    bnp = [mean.data_ptr(), rstd.data_ptr(), sc.data_ptr(), sh.data_ptr()]
    part = torch.zeros((M // 16 + 1) * 2 * C, device=gpu)
    outs = []
    for kern in ("gemm", "stream"):
        out = torch.full((N, H, H, C), float("nan"), device=gpu, dtype=BF)
        bacc = torch.zeros(rep * 2 * C, device=gpu, dtype=torch.float64)
        if kern == "gemm":
            nat.conv_gemm(1, dz.data_ptr(), w.data_ptr(), out.data_ptr(), 0, 0, 0, 0, 0, 0, 0, 0,
                          g.as_list(), [x.data_ptr()] + bnp + [part.data_ptr()], [],
                          [bacc.data_ptr()], [], [], 0.997, ref.BN_EPS, 1, st)
        else:
            nat.bnd1x1(2, [dz.data_ptr(), w.data_ptr(), x.data_ptr(), 0, out.data_ptr()] + bnp +
                       [0, bacc.data_ptr()], M, C, K, st)
        torch.cuda.synchronize()
        outs.append((out, bacc.view(rep, 2, C).sum(0)))
    (o0, s0), (o1, s1) = outs
    torch.testing.assert_close(o1.float(), o0.float(), rtol=0, atol=0)
    scale_ = s0.abs().max().item() + 1.0
    assert (s1 - s0).abs().max().item() <= 1e-5 * scale_
    dxt = torch.zeros(N, H, H, C, device=gpu, requires_grad=True)
    ref.conv2d(dxt, w.float(), 1).backward(dz.float())
    assert _rel(o1, dxt.grad) < 1e-2
    xf, gf = x.float().reshape(-1, C), o1.float().reshape(-1, C)
    gg = gf * ((xf * sc + sh) > 0).float()
    torch.testing.assert_close(s1[0].float(), gg.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(s1[1].float(), (gg * (xf - mean) * rstd).sum(0), rtol=1e-4, atol=1e-2)
