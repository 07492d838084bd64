"""bench.py's driver contract on a host without a GPU (--device cpu: the fp32
PyTorch trainer over gloo -- a plumbing check, never a headline number)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra=None, timeout=300):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_self_spawns_ranks_and_reports_process_group():
    r = _bench(["--device", "cpu", "--gpus", "2", "--model", "cifar_resnet20", "--batch", "8",
                "--steps", "2", "--warmup", "1"], {"DTR_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["pg_world_size"] == 2 and out["dist_backend"] == "gloo"
    assert out["steps"] == 2 and out["warmup"] == 1 and out["value"] > 0
    assert out["config"]["global_batch"] == 8 and out["config"]["per_gpu_batch"] == 4
    assert out["config"]["parallelism"] == "dp2" and out["dtype"] == "fp32"
    assert out["config"]["env"].get("DTR_DIST_BACKEND") == "gloo"
    for key in ("metric", "unit", "ms_per_step", "higher_is_better", "scaling", "vs_baseline",
                "data", "config"):
        assert key in out


def test_bench_spawn_fails_when_a_rank_fails():
    # an indivisible global batch makes every rank exit non-zero
    r = _bench(["--device", "cpu", "--gpus", "2", "--model", "cifar_resnet20", "--batch", "7",
                "--steps", "1", "--warmup", "0"], {"DTR_DIST_BACKEND": "gloo"})
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_refuses_diagnostic_and_unsupported_modes():
    r = _bench(["--device", "cpu", "--steps", "1"], {"DTR_DIAG_SKIP": "wgrad"})
    assert r.returncode == 2 and "DTR_DIAG_SKIP" in r.stderr
    r = _bench(["--gpus", "2", "--graph"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2 and "--graph" in r.stderr
    r = _bench(["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2
