"""Multi-rank data parallelism of the GPU engine, rehearsed on the one-GPU box.

RCCL refuses two ranks on one device, so these runs use DTR_DIST_BACKEND=gloo
(CUDA tensors, host-staged) with both ranks folded onto cuda:0.  What they pin
is the engine's DP logic: bucket cut points, all-reduce placement relative to
the side-stream weight gradients, broadcast-on-init, metric reduction, and the
bench.py multi-rank contract.  The RCCL/xGMI path itself runs in the driver's
8-GPU scaling bench."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _torchrun(args, port, timeout=600, extra_env=None):
    env = dict(os.environ, DTR_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.update(extra_env or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port)] + args
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


@pytest.mark.gpu
def test_dp_gradients_equal_sum_of_local_and_replicas_stay_identical(gpu):
    r = _torchrun(["scripts/dp_check.py"], 29711)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "DP_CHECK_OK" in r.stdout, r.stdout[-3000:]


@pytest.mark.gpu
def test_dp_reduce_groups_nested_in_buckets(gpu):
    # split-K reduce groups (DTR_REDUCE_MB) smaller than the all-reduce buckets:
    # several grouped reduces per bucket, the bucket joined after its last one
    r = _torchrun(["scripts/dp_check.py"], 29713,
                  extra_env={"DTR_REDUCE_MB": "0.05", "DP_CHECK_BUCKET_MB": "0.5"})
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "DP_CHECK_OK" in r.stdout, r.stdout[-3000:]


@pytest.mark.gpu
def test_dp_bf16_gradient_allreduce(gpu):
    # --allreduce_dtype bf16: buckets cast into a bf16 staging buffer, all-reduced, cast back
    r = _torchrun(["scripts/dp_check.py"], 29714, extra_env={"DP_CHECK_ALLREDUCE": "bf16"})
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "DP_CHECK_OK" in r.stdout, r.stdout[-3000:]


@pytest.mark.gpu
def test_bench_two_ranks_contract(gpu):
    r = _torchrun(["bench.py", "--gpus", "2", "--steps", "5", "--warmup", "2"], 29712)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 5 and out["config"]["global_batch"] == 128
    assert out["config"]["per_gpu_batch"] == 64 and out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0
