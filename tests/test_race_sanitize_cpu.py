"""Race detection and host sanitizers (SURVEY.md §5 "Race detection / sanitizers").

* the static stream-ordering check of the native plan (utils/streamcheck.py) on
  hand-built op lists: a sound fork/join passes, each class of race is reported;
* the native host code (csrc/host_io.cpp: the SSE4.2 CRC32C behind checkpoints,
  TFRecords and event files) built with AddressSanitizer + UBSan and run over
  unaligned, odd-length buffers, compared with the table implementation.
GPU ASan / XNACK are not available on the MI355X pool, so the GPU side is covered
by the plan check (the engine runs it on every plan it builds) and by the
bounds-asserting kernel tests in test_kernels_gpu.py.
"""
import os
import shutil
import subprocess

import pytest

from distributed_tensorflow_resnet_amd.utils import crc32c
from distributed_tensorflow_resnet_amd.utils.streamcheck import LAUNCH, RECORD, WAIT, check_plan_order

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "distributed_tensorflow_resnet_amd", "csrc")


def _plan(ops):
    """ops: list of (kind, stream, event) -> parallel lists."""
    return [o[0] for o in ops], [o[1] for o in ops], [o[2] for o in ops]


def _sound_step():
    # main: conv, record e0 | side: wait e0, wgrad, wgrad, record e1 | main: conv, wait e1
    return [(LAUNCH, 0, -1), (RECORD, 0, 0), (WAIT, 1, 0), (LAUNCH, 1, -1), (LAUNCH, 1, -1),
            (RECORD, 1, 1), (LAUNCH, 0, -1), (WAIT, 0, 1), (LAUNCH, 0, -1)]


def test_streamcheck_accepts_sound_fork_join():
    k, s, e = _plan(_sound_step())
    assert check_plan_order(k, s, e, [("bwd", 0, len(k))]) == []
    # main-only segments need no events at all
    k2, s2, e2 = _plan([(LAUNCH, 0, -1)] * 3)
    assert check_plan_order(k2, s2, e2, [("fwd", 0, 3)]) == []


def test_streamcheck_reports_missing_fork():
    ops = _sound_step()
    del ops[2]                      # side launches with no wait on main
    k, s, e = _plan(ops)
    errs = check_plan_order(k, s, e, [("bwd", 0, len(k))])
    assert any("(R2)" in x for x in errs), errs


def test_streamcheck_reports_missing_join():
    ops = _sound_step()[:-2] + [(LAUNCH, 0, -1)]   # main never waits on e1
    k, s, e = _plan(ops)
    errs = check_plan_order(k, s, e, [("bwd", 0, len(k))])
    assert any("(R3)" in x for x in errs), errs


def test_streamcheck_reports_late_side_work_and_bad_waits():
    ops = _sound_step() + [(LAUNCH, 1, -1)]        # side work after the join
    k, s, e = _plan(ops)
    assert any("(R3)" in x for x in check_plan_order(k, s, e, [("bwd", 0, len(k))]))
    # wait before the record / on an event of its own stream
    k, s, e = _plan([(WAIT, 1, 0), (RECORD, 0, 0), (RECORD, 0, 1), (WAIT, 0, 1)])
    errs = check_plan_order(k, s, e, [("x", 0, 4)])
    assert sum("(R1" in x for x in errs) == 2, errs
    # a record from an earlier segment does not order a later segment
    ops = _sound_step()
    k, s, e = _plan(ops)
    errs = check_plan_order(k, s, e, [("fwd", 0, 2), ("bwd", 2, len(k))])
    assert any("(R1)" in x for x in errs), errs
    with pytest.raises(ValueError):
        check_plan_order([0], [0, 1], [0], [])


_DRIVER = r"""
#include <stdint.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
namespace dtr { uint32_t crc32c_extend(uint32_t crc, const uint8_t* p, size_t n); }
int main(int argc, char** argv) {
  // exact-size heap copies so ASan flags any read past the end
  unsigned seed = 12345u;
  for (int len = 0; len <= 200; ++len) {
    for (int off = 0; off < 8; ++off) {
      uint8_t* buf = (uint8_t*)malloc((size_t)off + (size_t)len + (off + len == 0));
      for (int i = 0; i < off + len; ++i) { seed = seed * 1103515245u + 12345u; buf[i] = seed >> 16; }
      uint32_t c = dtr::crc32c_extend(0, buf + off, (size_t)len);
      if (off == 0) {
        printf("%d", len);
        for (int i = 0; i < len; ++i) printf(" %u", buf[i]);
        printf(" : %u\n", c);
      }
      free(buf);
    }
  }
  return 0;
}
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
@pytest.mark.parametrize("variant", ["native", "portable"])
def test_host_crc32c_under_asan_ubsan(tmp_path, variant):
    """Both CRC32C paths of host_io.cpp: SSE4.2 (x86) and the slicing-by-8 table
    every other host uses (forced here with DTR_CRC32C_PORTABLE)."""
    drv = tmp_path / "drv.cpp"
    drv.write_text(_DRIVER)
    exe = tmp_path / "crc_asan"
    cmd = ["g++", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", str(drv), os.path.join(CSRC, "host_io.cpp"), "-o", str(exe)]
    if variant == "portable":
        cmd.insert(1, "-DDTR_CRC32C_PORTABLE")
    r = subprocess.run(cmd, capture_output=True, text=True)
    err = r.stderr.lower()
    if r.returncode != 0 and ("asan" in err or "sanitizer" in err or "target" in err
                              or "unrecognized" in err):
        pytest.skip("sanitizer runtime / target not available: " + r.stderr[-200:])
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 201
    for ln in lines:
        head, crc = ln.split(" : ")
        vals = [int(v) for v in head.split()]
        assert crc32c._py_extend(0, bytes(vals[1:])) == int(crc)


# ---- three-stream plans: comm-stream all-reduces and host split points (R4) ----
def _names(n, at):
    out = ["k"] * n
    for i in at:
        out[i] = "all_reduce"
    return out


def _comm_step():
    # main: conv, record e0 | side: wait e0, wgrad, record e1 | main: wait e1, record e2 |
    # comm: wait e2, all_reduce, record e3 | main: conv, wait e3
    return [(LAUNCH, 0, -1), (RECORD, 0, 0), (WAIT, 1, 0), (LAUNCH, 1, -1), (RECORD, 1, 1),
            (WAIT, 0, 1), (RECORD, 0, 2), (WAIT, 2, 2), (LAUNCH, 2, -1), (RECORD, 2, 3),
            (LAUNCH, 0, -1), (WAIT, 0, 3)]


def test_streamcheck_comm_stream_sound_and_races():
    ops = _comm_step()
    k, s, e = _plan(ops)
    assert check_plan_order(k, s, e, [("bwd", 0, len(k))], names=_names(len(k), [8])) == []
    # the side stream is not joined before the all-reduce reads the bucket: R4
    bad = [o for i, o in enumerate(ops) if i != 5]
    k, s, e = _plan(bad)
    errs = check_plan_order(k, s, e, [("bwd", 0, len(k))], names=_names(len(k), [7]))
    assert any("(R4)" in x and "all_reduce" in x for x in errs), errs
    # the comm stream is never joined back: R3
    k, s, e = _plan(ops[:-1])
    errs = check_plan_order(k, s, e, [("bwd", 0, len(k))], names=_names(len(k), [8]))
    assert any("(R3)" in x and "stream-2" in x for x in errs), errs
    # an all-reduce launched without a fork from the main stream: R2
    k, s, e = _plan([(LAUNCH, 0, -1), (LAUNCH, 2, -1), (RECORD, 2, 0), (WAIT, 0, 0)])
    errs = check_plan_order(k, s, e, [("bwd", 0, 4)], names=_names(4, [1]))
    assert any("(R2)" in x for x in errs), errs


def test_streamcheck_device_dependency_orders_bucket_wait():
    """Persistent overlap plan: the comm stream's bucket all-reduce is ordered after the
    backward launch on the main stream by a device-side counter wait, not an event."""
    # main: fwd, record e0 | comm: wait e0, head | main: bwd (4) | comm: bucket wait (5),
    # all_reduce (6), record e1 | main: wait e1, optimizer
    ops = [(LAUNCH, 0, -1), (RECORD, 0, 0), (WAIT, 2, 0), (LAUNCH, 2, -1), (LAUNCH, 0, -1),
           (LAUNCH, 2, -1), (LAUNCH, 2, -1), (RECORD, 2, 1), (WAIT, 0, 1), (LAUNCH, 0, -1)]
    k, s, e = _plan(ops)
    seg = [("bwd", 0, len(k))]
    names = _names(len(k), [6])
    assert check_plan_order(k, s, e, seg, names=names, device_deps={5: 4}) == []
    # without the declared dependency the all-reduce races the backward: R4
    errs = check_plan_order(k, s, e, seg, names=names)
    assert any("(R4)" in x and "all_reduce" in x for x in errs), errs
    # a dependency on a later op, on an op of the same stream, or on a non-launch is refused
    for dep in ({5: 6}, {5: 3}, {5: 1}):
        errs = check_plan_order(k, s, e, seg, names=names, device_deps=dep)
        assert any("device dependency" in x for x in errs), (dep, errs)


def test_streamcheck_partial_device_dependency_holds_ops_to_covered_buffers():
    """a bucket wait orders the comm stream after the backward launch's COVERED
    buffers only (the bucket's gradients and parameters): the ops after it must declare
    their buffers and stay inside the coverage until an event orders the stream after
    the whole launch (R5); the all-reduce satisfies R4 only through that coverage."""
    # main: fwd, record e0 | comm: wait e0, head | main: bwd (4) | comm: bucket wait (5),
    # pack (6), all_reduce (7), update (8), record e1 | main: wait e1, optimizer
    ops = [(LAUNCH, 0, -1), (RECORD, 0, 0), (WAIT, 2, 0), (LAUNCH, 2, -1), (LAUNCH, 0, -1),
           (LAUNCH, 2, -1), (LAUNCH, 2, -1), (LAUNCH, 2, -1), (LAUNCH, 2, -1), (RECORD, 2, 1),
           (WAIT, 0, 1), (LAUNCH, 0, -1)]
    k, s, e = _plan(ops)
    seg = [("bwd", 0, len(k))]
    names = _names(len(k), [7])
    dep = {5: (4, {"grad:0", "param:0", "lr"})}
    good = {6: {"grad:0"}, 7: {"grad:0"}, 8: {"grad:0", "param:0", "lr"}}
    assert check_plan_order(k, s, e, seg, names=names, device_deps=dep, op_buffers=good) == []
    # an update of a parameter the backward may still read (a misassigned bucket): R5
    bad = {**good, 8: {"grad:0", "param:1"}}
    errs = check_plan_order(k, s, e, seg, names=names, device_deps=dep, op_buffers=bad)
    assert any("(R5)" in x and "param:1" in x for x in errs), errs
    # an op with no declared buffers beside the running producer: R5
    errs = check_plan_order(k, s, e, seg, names=names, device_deps=dep,
                            op_buffers={7: {"grad:0"}, 8: {"grad:0"}})
    assert any("(R5)" in x and "without declaring" in x for x in errs), errs
    # the all-reduce of a range the waits do not cover races the backward: R4
    errs = check_plan_order(k, s, e, seg, names=names, device_deps=dep,
                            op_buffers={**good, 7: {"grad:1"}})
    assert any("(R4)" in x and "all_reduce" in x for x in errs), errs
    # a second bucket wait widens the coverage
    dep2 = {5: (4, {"grad:0"}), 6: (4, {"grad:1", "param:1"})}
    ok2 = {7: {"grad:1"}, 8: {"grad:0", "param:1"}}
    assert check_plan_order(k, s, e, seg, names=names, device_deps=dep2, op_buffers=ok2) == []


def test_streamcheck_host_split_needs_join():
    """gloo rehearsal: the host all-reduces between Plan.run calls at a split index;
    a side-stream launch queued before the split but joined only later is a race
    the per-segment R3 cannot see."""
    ops = _sound_step()   # join (wait e1) at index 7
    k, s, e = _plan(ops)
    assert check_plan_order(k, s, e, [("bwd", 0, len(k))], barriers=[8]) == []
    errs = check_plan_order(k, s, e, [("bwd", 0, len(k))], barriers=[6])
    assert any("(R4)" in x and "host all-reduce split" in x for x in errs), errs
