"""Shape fuzzing of the conv kernels (hypothesis over the Appendix-A shape
space) against the plain-PyTorch fp32 reference (ops/reference.py): forward, data
gradient and weight gradient over random batch / spatial size / channels / kernel /
stride, including partial tiles and the direct-kernel shapes; plus the fp64
BatchNorm accumulators (GemmArgs::stat_acc / bnb_acc) against torch reductions of
the kernel's own output.  Derandomized, so a failure reproduces."""
import math

import pytest
import torch

hyp = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as st  # noqa: E402

from distributed_tensorflow_resnet_amd.ops import functional as fn  # noqa: E402
from distributed_tensorflow_resnet_amd.ops import reference as ref  # noqa: E402

pytestmark = pytest.mark.gpu
BF = torch.bfloat16
SETTINGS = dict(max_examples=24, deadline=None, derandomize=True)


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


shapes = st.tuples(
    st.integers(1, 4),                               # N
    st.integers(3, 20),                              # H = W
    st.sampled_from([8, 16, 24, 32, 64, 96, 128]),   # C (multiple of 8)
    st.sampled_from([16, 32, 48, 64, 128, 256]),     # K (multiple of 16)
    st.sampled_from([1, 3]),                         # kernel
    st.sampled_from([1, 2]),                         # stride
)


def _operands(gpu, N, H, C, K, k, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(N, H, H, C, generator=g).to(gpu, BF)
    w = (torch.randn(k, k, C, K, generator=g) / math.sqrt(k * k * C)).to(gpu, BF)
    return x, w


@settings(**SETTINGS)
@given(shapes)
def test_fuzz_conv_fwd(gpu, shape):
    N, H, C, K, k, s = shape
    x, w = _operands(gpu, N, H, C, K, k, 11)
    y = fn.conv2d_fwd(x, w.permute(3, 0, 1, 2).contiguous(), s)
    r = ref.conv2d(x.float(), w.float(), s)
    assert y.shape == r.shape
    assert _rel(y, r) < 1e-2, shape


# dgrad writes C output channels: the kernels need C % 16 == 0 (the 3-channel stem
# input, padded to 8, never takes a data gradient)
dgrad_shapes = shapes.filter(lambda t: t[2] % 16 == 0)


@settings(**SETTINGS)
@given(dgrad_shapes)
def test_fuzz_conv_dgrad(gpu, shape):
    N, H, C, K, k, s = shape
    x, w = _operands(gpu, N, H, C, K, k, 12)
    xf = x.float().requires_grad_(True)
    r = ref.conv2d(xf, w.float(), s)
    dy = torch.randn(r.shape, generator=torch.Generator().manual_seed(3)).to(gpu, BF)
    r.backward(dy.float())
    dx = fn.conv2d_dgrad(dy, w.contiguous(), tuple(x.shape), s)
    assert _rel(dx, xf.grad) < 1e-2, shape


@settings(**SETTINGS)
@given(shapes)
def test_fuzz_conv_wgrad(gpu, shape):
    N, H, C, K, k, s = shape
    x, _ = _operands(gpu, N, H, C, K, k, 13)
    w = torch.zeros(k, k, C, K, device=gpu, requires_grad=True)
    r = ref.conv2d(x.float(), w, s)
    dy = torch.randn(r.shape, generator=torch.Generator().manual_seed(4)).to(gpu, BF)
    r.backward(dy.float())
    dw = fn.conv2d_wgrad(dy, x, k, k, s)
    assert _rel(dw, w.grad) < 1e-2, shape


@settings(**SETTINGS)
@given(shapes, st.booleans())
def test_fuzz_bn_stat_accumulators(gpu, shape, shifted):
    """Output BN statistics through the fp64 accumulator replicas == torch mean/var of
    the bf16 output (also with a large common offset: E[y^2] - mean^2 in fp64)."""
    N, H, C, K, k, s = shape
    nat = fn.native()
    x, w = _operands(gpu, N, H, C, K, k, 14)
    g = fn.ConvGeom(N, H, H, C, K, k, k, s)
    M = N * g.Ho * g.Wo
    tiles, _ = fn.stat_tiles(M, K)
    part = torch.empty(tiles * 2 * K, device=gpu)
    acc = torch.zeros(nat.bn_acc_rep() * 2 * K, dtype=torch.float64, device=gpu)
    res = (torch.full((N, g.Ho, g.Wo, K), 8.0, device=gpu).to(BF) if shifted else None)
    y = fn.conv2d_fwd(x, w.permute(3, 0, 1, 2).contiguous(), s, residual=res, stat_part=part,
                      fin=[acc])
    gamma, beta = torch.ones(K, device=gpu), torch.zeros(K, device=gpu)
    mm, mv = torch.zeros(K, device=gpu), torch.ones(K, device=gpu)
    mean, rstd, _, _ = fn.bn_finalize(acc, -1, 0, M, gamma, beta, mm, mv)
    yf = y.float().reshape(M, K)
    var = yf.var(0, unbiased=False)
    assert _rel(mean, yf.mean(0)) < 1e-4, shape
    assert _rel(1.0 / rstd ** 2 - 1.001e-5, var) < 1e-3, shape
