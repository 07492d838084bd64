"""The MLP debug model's synchronous data parallelism (reference logist_model.py:62-86:
Adam under SyncReplicasOptimizer) on 2 gloo CPU ranks: the replicas stay identical and
follow the single-process model trained on the whole batch."""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data(n=8):
    g = torch.Generator().manual_seed(7)
    return torch.randn(2 * n, 3, 8, 8, generator=g), torch.randint(0, 10, (2 * n,), generator=g)


def _rank(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from distributed_tensorflow_resnet_amd.models.resnet_model import HParams
    from distributed_tensorflow_resnet_amd.parallel.dist import DistContext
    from logist_model import LRNet

    ctx = DistContext(backend="gloo")
    x, y = _data()
    n = x.shape[0] // world
    xs, ys = x[rank * n:(rank + 1) * n], y[rank * n:(rank + 1) * n]
    hps = HParams(num_classes=10, lrn_rate=0.01, weight_decay_rate=0.0, optimizer="adam")
    m = LRNet(hps, xs, ys, "train", seed=100 + rank, dist_ctx=ctx)   # different inits
    for _ in range(3):
        m.build_graph()
        m.train_op()
    torch.save([p.detach().clone() for p in m.params], os.path.join(out_dir, f"r{rank}.pt"))
    ctx.shutdown()


def test_mlp_sync_replicas_two_gloo_ranks(tmp_path):
    from distributed_tensorflow_resnet_amd.models.resnet_model import HParams
    from logist_model import LRNet

    mp.spawn(_rank, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    for a, b in zip(r0, r1):
        assert torch.equal(a, b)   # broadcast init + identical averaged updates
    x, y = _data()
    hps = HParams(num_classes=10, lrn_rate=0.01, weight_decay_rate=0.0, optimizer="adam")
    ref = LRNet(hps, x, y, "train", seed=100)   # rank 0's init, the whole batch
    for _ in range(3):
        ref.build_graph()
        ref.train_op()
    for a, b in zip(r0, ref.params):
        assert torch.allclose(a, b.detach(), atol=1e-5, rtol=1e-4)
