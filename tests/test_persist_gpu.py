"""Persistent multi-layer prototype (csrc/persist.hip): L chained CIFAR stage-3 convs in
one launch with grid barriers == the PyTorch fp32 reference of the same chain
(batch-statistics BN between layers, residual on every second conv, bf16 rounding where
the kernel rounds); repeated launches reuse nothing but the weights."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "scripts"))


@pytest.mark.parametrize("N,L", [(4, 4), (16, 6), (32, 16)])
def test_persistent_stage_matches_reference(gpu, N, L):
    import persist_probe as pp

    from distributed_tensorflow_resnet_amd.ops import functional as fn

    nat = fn.native()
    ins = pp.make_inputs(N, L, gpu, seed=N + L)
    ref = pp.reference(*ins)
    for _ in range(2):
        y, _ = pp.run_persistent(nat, *ins)
        for i in range(L):
            rel = ((y[i].float() - ref[i].float()).norm() / ref[i].float().norm()).item()
            assert rel < 2e-2, f"layer {i}: rel err {rel}"
