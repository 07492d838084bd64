"""MLP baseline model (reference logist_model.py:10-86, `LRNet`): one hidden
layer of `hidden_units` (default 100) ReLU units over flattened images, softmax
cross-entropy, Adam.  A debugging model in the reference (its use is commented
out at resnet_cifar_main.py:271); kept for parity on the CPU path.

Distributed (``dist_ctx`` with world > 1): the reference wraps Adam in
SyncReplicasOptimizer (logist_model.py:62-86) -- every step applies the average of
all replicas' gradients.  Here the replicas start from rank 0's parameters
(broadcast) and all-reduce (average) their gradients before the same Adam step, so
they stay identical: synchronous data parallelism without a parameter server.
"""
import torch
import torch.nn.functional as F

HIDDEN_UNITS = 100


class LRNet:
    def __init__(self, hps, images, labels, mode, hidden_units=HIDDEN_UNITS, seed=0,
                 dist_ctx=None):
        self.hps = hps
        self.images = images
        self.labels = labels
        self.mode = mode
        g = torch.Generator().manual_seed(seed)
        d = int(images[0].numel())
        nc = hps.num_classes
        self.w1 = (torch.randn(d, hidden_units, generator=g) / d ** 0.5).requires_grad_()
        self.b1 = torch.zeros(hidden_units, requires_grad=True)
        self.w2 = (torch.randn(hidden_units, nc, generator=g) / hidden_units ** 0.5).requires_grad_()
        self.b2 = torch.zeros(nc, requires_grad=True)
        self.params = [self.w1, self.b1, self.w2, self.b2]
        self.dist = dist_ctx if dist_ctx is not None and dist_ctx.world_size > 1 else None
        if self.dist is not None:   # every replica starts from rank 0's parameters
            with torch.no_grad():
                for p in self.params:
                    self.dist.broadcast(p.data, 0)
        self.opt = torch.optim.Adam(self.params, lr=hps.lrn_rate)
        self.global_step = 0

    def build_graph(self, istrain=True):
        x = self.images.reshape(self.images.shape[0], -1).float()
        h = torch.relu(x @ self.w1 + self.b1)
        self.logits = h @ self.w2 + self.b2
        self.predictions = torch.softmax(self.logits, 1)
        y = self.labels.argmax(1) if self.labels.dim() == 2 else self.labels
        self.cost = F.cross_entropy(self.logits, y.long())
        return self

    def train_op(self):
        self.opt.zero_grad()
        self.cost.backward()
        if self.dist is not None:   # SyncReplicasOptimizer: the replicas' mean gradient
            flat = torch.cat([p.grad.reshape(-1) for p in self.params])
            self.dist.all_reduce_sum(flat)
            flat /= self.dist.world_size
            off = 0
            for p in self.params:
                n = p.numel()
                p.grad.copy_(flat[off:off + n].view_as(p.grad))
                off += n
        self.opt.step()
        self.global_step += 1
        return self.global_step
