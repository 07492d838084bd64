"""Space-to-depth ImageNet stem (csrc/data.hip stem_s2d_*, Engine.stem_s2d): the
7x7 / stride-2 conv with TF fixed padding (resnet_model_official.py:80-91, the
stem of imagenet_resnet_v2_generator) computed as a 4x4 / stride-1 conv over the
[N, H/2, W/2, 16] space-to-depth image.  Checked against an fp32 PyTorch conv of
the same op (forward and weight gradient), and the engine with and without it."""
import pytest
import torch
import torch.nn.functional as F

from distributed_tensorflow_resnet_amd import native
from distributed_tensorflow_resnet_amd.models.spec import imagenet_spec
from distributed_tensorflow_resnet_amd.train.engine import Engine, imagenet_lr_schedule

pytestmark = pytest.mark.gpu


def _s2d(x):
    """[N, H, W, 3] -> [N, H/2, W/2, 16], channel (rh*2 + rw)*4 + c (c = 3 zero)."""
    N, H, W, C = x.shape
    xp = torch.zeros(N, H, W, 4, dtype=x.dtype, device=x.device)
    xp[..., :C] = x
    return xp.view(N, H // 2, 2, W // 2, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(
        N, H // 2, W // 2, 16).contiguous()


def _rel(a, b):
    return ((a - b).norm() / b.norm()).item()


@pytest.mark.parametrize("N,H", [(4, 32), (2, 224)])
def test_stem_s2d_conv_matches_7x7_stride2(gpu, N, H):
    nat = native(required=True)
    K = 64
    torch.manual_seed(0)
    x = torch.randn(N, H, H, 3, device=gpu).to(torch.bfloat16)
    w7 = torch.randn(7, 7, 3, K, device=gpu) * 0.1            # HWIO fp32 master
    st = torch.cuda.current_stream().cuda_stream
    w4 = torch.empty(K * 256, dtype=torch.bfloat16, device=gpu)
    nat.stem_s2d_pack(w7.data_ptr(), w4.data_ptr(), K, st)
    xs = _s2d(x)
    Ho = H // 2
    geom = [N, Ho, Ho, 16, Ho, Ho, K, 4, 4, 1, 2]
    y = torch.empty(N, Ho, Ho, K, dtype=torch.bfloat16, device=gpu)
    nat.conv_gemm(0, xs.data_ptr(), w4.data_ptr(), y.data_ptr(), 0, 0, 0, 0, 0, 0, 0, 0, geom,
                  [], [], [], [], [], 0.997, 1e-5, 1, st)
    # fp32 reference: explicit TF padding (3, 3) then a VALID 7x7 / 2 conv
    xr = x.float().permute(0, 3, 1, 2)
    wv = w7.to(torch.bfloat16).float().permute(3, 2, 0, 1).clone().requires_grad_(True)
    ref = F.conv2d(F.pad(xr, (3, 3, 3, 3)), wv, stride=2)
    torch.cuda.synchronize()
    assert _rel(y.float(), ref.permute(0, 2, 3, 1)) < 1e-2
    # weight gradient: split-K wgrad over the s2d operands, 4x4x16 reduce, map to 7x7x3
    dy = torch.randn(N, Ho, Ho, K, device=gpu).to(torch.bfloat16)
    sp, pps = nat.wgrad_pick_splits(geom)
    part = torch.empty(sp * K * 256, device=gpu)
    nat.conv_wgrad(dy.data_ptr(), xs.data_ptr(), 0, 0, part.data_ptr(), geom, sp, pps, st)
    g4 = torch.empty(256 * K, device=gpu)
    nat.wgrad_reduce(part.data_ptr(), g4.data_ptr(), sp, K, K, 16, 16, 16, 1.0, 0, st)
    g7 = torch.full((7, 7, 3, K), float("nan"), device=gpu)
    nat.stem_s2d_grad(g4.data_ptr(), g7.data_ptr(), K, st)
    ref.backward(dy.float().permute(0, 3, 1, 2))
    torch.cuda.synchronize()
    assert torch.isfinite(g7).all()
    assert _rel(g7, wv.grad.permute(2, 3, 1, 0)) < 1e-2


def _engine(spec, monkeypatch, gpu, s2d, imgs, labels, master, stats):
    monkeypatch.setenv("DTR_TUNE", f"stem_s2d={int(s2d)}")
    eng = Engine(spec, imgs.shape[0], weight_decay=1e-4, lr_schedule=imagenet_lr_schedule(),
                 device=gpu, input_mode="nhwc", use_graph=False)
    assert eng.stem_s2d == s2d
    if master is not None:
        eng.params.master.copy_(master)
        eng.params.stats.copy_(stats)
        eng.repack()
    eng.set_batch(imgs, labels)
    st = torch.cuda.current_stream().cuda_stream
    eng.forward_backward(st)
    torch.cuda.synchronize()
    return eng


def test_engine_stem_s2d_matches_direct_stem(gpu, monkeypatch):
    spec = imagenet_spec(0, num_classes=10, image_hw=64, block="bottleneck", layers=[1, 1, 1, 1])
    torch.manual_seed(1)
    imgs = torch.randn(8, 64, 64, 3, device=gpu)
    labels = torch.randint(0, 10, (8,), device=gpu)
    a = _engine(spec, monkeypatch, gpu, False, imgs, labels, None, None)
    b = _engine(spec, monkeypatch, gpu, True, imgs, labels, a.params.master, a.params.stats)
    # same network input, laid out for each stem
    assert torch.equal(b.x_in.float(), _s2d(a.x_in[..., :3]).float())
    assert torch.equal(a.stem_out, b.stem_out) or _rel(b.stem_out.float(), a.stem_out.float()) < 1e-2
    la, lb = a.scalars[0].item(), b.scalars[0].item()
    assert abs(la - lb) < 1e-2 * max(1.0, abs(la))
    s = a.params.slot(f"{spec.stem.name}/kernel")
    ga, gb = a.grad[s.offset:s.offset + s.numel], b.grad[s.offset:s.offset + s.numel]
    print("stem grad rel", _rel(gb, ga), "all", _rel(b.grad, a.grad))
    assert torch.nn.functional.cosine_similarity(ga, gb, dim=0).item() > 0.98
    assert _rel(gb, ga) < 0.1
