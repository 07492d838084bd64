"""The native Plan executor's multi-threaded issue (bindings.cpp Plan::run): each
stream's ops are issued by their own host thread and a cross-stream wait only after
the matching record was issued in the same run -- so the device-side ordering of a
fork/join chain must be exactly the single-threaded one, run after run."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _chain(nat, a, b, c, n, rounds):
    """main: fill a = k; fork -> side: b = bf16(a); join -> main: c = f32(b); repeated,
    with the comm stream (2) doing its own fork/join on the way."""
    p = nat.Plan()
    for k in range(rounds):
        p.use_stream(0)
        p.fill(a.data_ptr(), n, float(k + 1))
        e1 = p.new_event()
        p.record(e1)
        p.use_stream(1)
        p.wait(e1)
        p.cast_f32_bf16(a.data_ptr(), b.data_ptr(), n)
        e2 = p.new_event()
        p.record(e2)
        p.use_stream(2)
        p.wait(e2)
        p.cast_bf16_f32(b.data_ptr(), c[k].data_ptr(), n)
        e3 = p.new_event()
        p.record(e3)
        p.use_stream(0)
        p.wait(e3)
    return p


@pytest.mark.parametrize("threaded", [True, False])
def test_threaded_issue_keeps_fork_join_order(gpu, threaded):
    import distributed_tensorflow_resnet_amd as dtr

    nat = dtr.native(required=True)
    n, rounds = 1 << 20, 24
    a = torch.zeros(n, device=gpu)
    b = torch.zeros(n, dtype=torch.bfloat16, device=gpu)
    c = torch.zeros(rounds, n, device=gpu)
    p = _chain(nat, a, b, c, n, rounds)
    p.set_threaded(threaded)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    st = torch.cuda.current_stream()
    for rep in range(20):
        c.zero_()
        p.run(0, p.size(), st.cuda_stream, s1.cuda_stream, s2.cuda_stream)
        torch.cuda.synchronize()
        want = torch.arange(1, rounds + 1, device=gpu, dtype=torch.float32)
        assert torch.equal(c[:, 0], want) and torch.equal(c[:, -1], want), rep
