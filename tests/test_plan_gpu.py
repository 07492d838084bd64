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


def test_splitk_workspace_is_per_stream(gpu):
    """Two split-K convs recorded on two streams of one plan: each
    stream brings its own plan-owned workspace, so running them concurrently gives
    bitwise the result of running them one after the other."""
    import distributed_tensorflow_resnet_amd as dtr

    nat = dtr.native(required=True)
    N, H, C, K = 16, 7, 512, 512
    geom = [N, H, H, C, H, H, K, 3, 3, 1, 1]
    assert nat.conv_gemm_splitk_bytes(0, geom) > 0, "shape must take the split-K loop"
    g = torch.Generator(device="cpu").manual_seed(0)
    xs = [torch.randn(N, H, H, C, generator=g).to(torch.bfloat16).to(gpu) for _ in range(2)]
    ws = [(torch.randn(K, 3, 3, C, generator=g) * 0.05).to(torch.bfloat16).to(gpu) for _ in range(2)]
    outs = [torch.zeros(N, H, H, K, dtype=torch.bfloat16, device=gpu) for _ in range(2)]

    def conv(p, i):
        p.conv_gemm(0, xs[i].data_ptr(), ws[i].data_ptr(), outs[i].data_ptr(), 0, 0, 0, 0, 0, 0,
                    0, 0, geom, [], [], [], [], [], 0.997, 1e-5, 1)

    seq = nat.Plan()
    conv(seq, 0)
    conv(seq, 1)
    st = torch.cuda.current_stream().cuda_stream
    seq.run(0, seq.size(), st)
    torch.cuda.synchronize()
    ref = [o.clone() for o in outs]
    par = nat.Plan()
    ev = par.new_event()
    par.record(ev)
    par.use_stream(1)
    par.wait(ev)
    conv(par, 1)
    j = par.new_event()
    par.record(j)
    par.use_stream(0)
    conv(par, 0)
    par.wait(j)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(10):
        for o in outs:
            o.zero_()
        par.run(0, par.size(), st, s1.cuda_stream, s2.cuda_stream)
        torch.cuda.synchronize()
        assert torch.equal(outs[0], ref[0]) and torch.equal(outs[1], ref[1])
