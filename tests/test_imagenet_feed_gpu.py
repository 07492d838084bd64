"""Real-data ImageNet feed, device half: imagenet_u8_pack (csrc/data.hip) turns
the workers' uint8 HWC crops into the stem's bf16 NHWC-8 operand with the VGG
random flip and mean subtraction (vgg_preprocessing.py:37-39, 284-314), and the
engine's imagenet_u8 input mode trains from it."""
import pytest
import torch

from distributed_tensorflow_resnet_amd.models.spec import imagenet_spec
from distributed_tensorflow_resnet_amd.train.engine import Engine, imagenet_lr_schedule

pytestmark = pytest.mark.gpu
MEANS = torch.tensor([123.68, 116.78, 103.94])


def test_u8_pack_flip_and_mean(gpu):
    import distributed_tensorflow_resnet_amd as dtr

    nat = dtr.native(required=True)
    N, H, W = 16, 20, 24
    img = torch.randint(0, 256, (N, H, W, 3), dtype=torch.uint8, device=gpu)
    out = torch.full((N, H, W, 8), 7.0, dtype=torch.bfloat16, device=gpu)
    gstep = torch.tensor([5], dtype=torch.int64, device=gpu)
    zero = torch.ones(64, device=gpu)
    st = torch.cuda.current_stream().cuda_stream
    nat.imagenet_u8_pack(img.data_ptr(), out.data_ptr(), N, H, W, 99, gstep.data_ptr(), 1,
                         zero.data_ptr(), zero.numel() * 4, 0, st)
    torch.cuda.synchronize()
    assert torch.count_nonzero(zero) == 0
    assert torch.count_nonzero(out[..., 3:]) == 0
    ref = (img.float().cpu() - MEANS).to(torch.bfloat16).float()
    got = out[..., :3].float().cpu()
    flips = 0
    for n in range(N):
        if torch.equal(got[n], ref[n]):
            continue
        assert torch.equal(got[n], ref[n].flip(1)), n
        flips += 1
    assert 2 <= flips <= N - 2          # a fair coin per image
    # eval (train=0): no flip; a different step reshuffles the flips
    nat.imagenet_u8_pack(img.data_ptr(), out.data_ptr(), N, H, W, 99, gstep.data_ptr(), 0, 0, 0, 0, st)
    torch.cuda.synchronize()
    assert torch.equal(out[..., :3].float().cpu(), ref)
    # space-to-depth stem operand: [N][H/2][W/2][(rh*2 + rw)*4 + c], c = 3 zero
    s2d = torch.full((N, H // 2, W // 2, 16), 7.0, dtype=torch.bfloat16, device=gpu)
    nat.imagenet_u8_pack(img.data_ptr(), s2d.data_ptr(), N, H, W, 99, gstep.data_ptr(), 0, 0, 0, 1,
                         st)
    torch.cuda.synchronize()
    r4 = torch.zeros(N, H, W, 4)
    r4[..., :3] = ref
    want = r4.view(N, H // 2, 2, W // 2, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(N, H // 2, W // 2, 16)
    assert torch.equal(s2d.float().cpu(), want)


def test_engine_trains_from_u8_crops(gpu):
    spec = imagenet_spec(0, num_classes=10, image_hw=64, block="bottleneck", layers=[1, 1, 1, 1])
    eng = Engine(spec, 8, weight_decay=1e-4, lr_schedule=imagenet_lr_schedule(), device=gpu,
                 input_mode="imagenet_u8")
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 256, (8, 64, 64, 3), generator=g, dtype=torch.uint8).pin_memory()
    y = torch.randint(0, 10, (8,), generator=g)
    eng.set_batch(x, y)
    losses = []
    for _ in range(12):
        eng.step()
        losses.append(eng.metrics()["cross_entropy"])
    assert int(eng.gstep.item()) == 12
    assert all(torch.isfinite(torch.tensor(losses)))
    assert min(losses[-3:]) < losses[0]     # memorises the fixed batch


def test_eval_short_last_batch(gpu):
    """The evaluator's static plan scores a short last batch (an eval loader's remainder:
    several workers over 390-image ImageNet validation shards) from the valid rows only:
    loss and correct count equal those rows' share of a full batch."""
    from distributed_tensorflow_resnet_amd.models.spec import cifar_spec
    from distributed_tensorflow_resnet_amd.train.evaluator import GPUInference

    torch.manual_seed(3)
    inf = GPUInference(cifar_spec(8), 8, device=gpu)
    x = torch.randn(8, 32, 32, 3) * 60 + 120
    y = torch.randint(0, 10, (8,))
    _, _, probs = inf.run(x, y)
    p = probs[:5].float().cpu()
    loss5, corr5, _ = inf.run(x[:5], y[:5])
    ref_loss = float(-torch.log(p.gather(1, y[:5, None]).clamp_min(1e-30)).sum())
    assert abs(loss5 - ref_loss) < 1e-3 * max(1.0, abs(ref_loss))
    assert corr5 == float((p.argmax(1) == y[:5]).sum())
