"""The shared-memory rehearsal transport of the native communicator
(csrc/comm_shm.cpp) on host memory, several real processes: the collective
core that the one-GPU box's world > 1 rehearsals run behind the same Comm
interface as RCCL.  Pins rank-order (bitwise predictable) sums for fp32 / fp64
/ bf16, chunking through a small slot, broadcast, the segment's cleanup, and the
failure paths the watchdog relies on: a dead peer, a timeout and a peer's abort
all fail the survivor fast with async_error() == 6 (ncclRemoteError)."""
import multiprocessing as mp
import os
import time
import uuid

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _nat():
    import sys

    sys.path.insert(0, ROOT)
    import distributed_tensorflow_resnet_amd as dtr

    nat = dtr.native(required=False)
    return nat


def _data(rank, n, dtype):
    rng = np.random.default_rng(100 + rank)
    x = (rng.standard_normal(n) * (rank + 1) * 1e3).astype(np.float32)
    if dtype == "bf16":
        return (x.view(np.uint32) >> 16).astype(np.uint16)   # truncated to bf16 bits
    return x.astype(np.float64) if dtype == "f64" else x


def _bf16_to_f32(b):
    return (b.astype(np.uint32) << 16).view(np.float32)


def _f32_to_bf16_rne(x):
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return u.astype(np.uint16)


def _worker(kind, name, world, rank, n, dtype, slot, q, extra):
    try:
        nat = _nat()
        code = {"f32": nat.COMM_F32, "f64": nat.COMM_F64, "bf16": nat.COMM_BF16}[dtype]
        timeout = extra.get("timeout", 30.0)
        comm = nat.Comm.shm(name, world, rank, -1, slot_bytes=slot, timeout_s=timeout,
                            init_timeout_s=120.0)
        assert comm.transport == "shm" and comm.world == world and comm.rank == rank
        if kind == "sum":
            x = _data(rank, n, dtype)
            comm.host_all_reduce(x.ctypes.data, n, code)
            b = _data(rank, n, dtype) if rank == 0 else np.zeros_like(_data(0, n, dtype))
            comm.host_broadcast(b.ctypes.data, n, code, 0)
            q.put((rank, "ok", x.tobytes(), b.tobytes(), os.path.exists("/dev/shm" + name)))
            return
        if kind in ("dead", "sleep", "abort"):
            x = _data(rank, n, dtype)
            if rank == 1:
                if kind == "dead":
                    os._exit(0)
                if kind == "abort":
                    comm.abort()
                    q.put((rank, "aborted", comm.async_error()))
                    time.sleep(2.0)
                    return
                time.sleep(extra.get("sleep", 5.0))
                q.put((rank, "slept", 0))
                return
            t0 = time.monotonic()
            try:
                comm.host_all_reduce(x.ctypes.data, n, code)
                q.put((rank, "no-error", 0.0, comm.async_error(), ""))
            except RuntimeError as e:
                q.put((rank, "raised", time.monotonic() - t0, comm.async_error(), str(e)))
            return
    except Exception as e:   # noqa: BLE001
        q.put((rank, "exception", repr(e)))


def _run(kind, world, n=1000, dtype="f32", slot=4096, extra=None, timeout=60):
    if _nat() is None:
        pytest.skip("native extension not built")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"/dtr-test-{uuid.uuid4().hex[:12]}"
    ps = [ctx.Process(target=_worker, args=(kind, name, world, r, n, dtype, slot, q, extra or {}))
          for r in range(world)]
    for p in ps:
        p.start()
    out = []
    deadline = time.time() + timeout
    while len(out) < world and time.time() < deadline:
        try:
            out.append(q.get(timeout=0.5))
        except Exception:   # noqa: BLE001 - queue.Empty
            if kind == "dead" and len(out) == world - 1:
                break
    for p in ps:
        p.join(timeout=10)
        if p.is_alive():
            p.kill()
    assert not os.path.exists("/dev/shm" + name), "segment left behind"
    return {o[0]: o for o in out}


@pytest.mark.parametrize("world,dtype,n,slot", [(2, "f32", 5000, 4096), (3, "f32", 777, 1 << 16),
                                               (2, "bf16", 9000, 4096), (3, "bf16", 500, 4096),
                                               (2, "f64", 1500, 4096)])
def test_shm_all_reduce_rank_order_sum_and_broadcast(world, dtype, n, slot):
    res = _run("sum", world, n, dtype, slot)
    assert sorted(res) == list(range(world)), res
    npdt = {"f32": np.float32, "f64": np.float64, "bf16": np.uint16}[dtype]
    xs = [_data(r, n, dtype) for r in range(world)]
    if dtype == "bf16":
        acc = _bf16_to_f32(xs[0])
        for x in xs[1:]:
            acc = (acc + _bf16_to_f32(x)).astype(np.float32)
        want = _f32_to_bf16_rne(acc)
    else:
        want = xs[0].copy()
        for x in xs[1:]:
            want = want + x
    for r in range(world):
        assert res[r][1] == "ok", res[r]
        got = np.frombuffer(res[r][2], dtype=npdt)
        assert np.array_equal(got, want), f"rank {r} differs from the rank-order sum"
        bc = np.frombuffer(res[r][3], dtype=npdt)
        assert np.array_equal(bc, xs[0]), f"rank {r}: broadcast from rank 0 differs"
        assert not res[r][4], "the segment name must be unlinked once every rank attached"


def test_shm_dead_peer_fails_survivor_fast():
    res = _run("dead", 2, extra={"timeout": 60.0})
    st, dt, err, msg = res[0][1], res[0][2], res[0][3], res[0][4]
    assert st == "raised", res
    assert dt < 10.0, f"dead peer detected only after {dt:.1f}s"
    assert err == 6 and "gone" in msg, (err, msg)


def test_shm_timeout_and_peer_abort():
    res = _run("sleep", 2, extra={"timeout": 1.0, "sleep": 4.0})
    assert res[0][1] == "raised" and 0.9 < res[0][2] < 3.5 and res[0][3] == 6, res
    assert "timed out" in res[0][4]
    res = _run("abort", 2, extra={"timeout": 60.0})
    assert res[1][1] == "aborted" and res[1][2] == 6, res
    assert res[0][1] == "raised" and res[0][2] < 10.0 and res[0][3] == 6, res
    assert "aborted by rank 1" in res[0][4]


def test_shm_init_times_out_without_peer():
    """A rank that never attaches: the others' construction fails (no hang)."""
    if _nat() is None:
        pytest.skip("native extension not built")
    nat = _nat()
    name = f"/dtr-test-{uuid.uuid4().hex[:12]}"
    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match="timed out"):
        nat.Comm.shm(name, 2, 0, -1, slot_bytes=4096, timeout_s=0.5)
    assert time.monotonic() - t0 < 5.0
    assert not os.path.exists("/dev/shm" + name)
    with pytest.raises(ValueError):
        nat.Comm.shm("no-slash", 2, 0, -1)
    with pytest.raises(ValueError):
        nat.Comm.shm(name, 2, 2, -1)
