"""Host-side stream-ordering check of a recorded native Plan (race detection).

The training step is a static list of ops on three HIP streams (main = 0,
side = 1 for weight gradients, comm = 2 for the RCCL all-reduces) ordered only
by event record/wait pairs (engine.py `_flush_side` / `_flush_buckets` /
`_emit_allreduce`).  A missing fork or join is a data race that no GPU
sanitizer on this pool can find (no XNACK / GPU ASan), and it usually shows up
only as rare, non-reproducible gradient corruption.  This module checks the op
list statically, once, when the engine builds the plan (SURVEY.md §5 "Race
detection": stream-ordering asserts around comm/compute events; the reference
has none -- its only checks are graph asserts,
`/root/reference/vgg_preprocessing.py:67-84`, `cifar_input.py:110-115`).

It is a check of the fork/join STRUCTURE only, with happens-before computed by
vector clocks over the three streams.  It does not know which buffers an op
reads or writes.  For example, a side-stream op that reads a buffer the main
stream rewrites after the side stream's last fork passes R2.  Buffer-level races
are the job of the dynamic check in utils/racecheck.py: it runs the plan under
randomly perturbed schedules and compares the state bitwise against plan order
on one stream.  The rules below are stated conservatively in terms of "all work
queued earlier".  Rules, per segment (a range of ops the host runs with one
`Plan.run` call):

R1  every wait names an event recorded earlier in the same segment, on another
    stream (a wait on a never-recorded event is a no-op: no ordering at all; a
    record from a previous segment may be a previous step's);
R2  fork: every side- or comm-stream launch follows a wait (directly or through
    another stream) on an event the main stream recorded in the same segment
    (otherwise it races with the work the host queued before the segment, e.g.
    the previous step's optimizer);
R3  join: everything a segment launched on the side and comm streams is ordered
    before the main stream's end of the segment (otherwise the next segment /
    optimizer reads gradients that are still being written or all-reduced);
R4  collectives: an all-reduce (or a host split point, `barriers`: an index
    where the host issues a c10d all-reduce on the main stream between two
    `Plan.run` calls) is ordered after EVERY launch queued before it in the
    plan, on every stream -- the bucket it reads is complete, whichever stream
    produced its gradients.
R5  partial device dependencies: see below.

Device-side dependencies (`device_deps` {op: producer op} or {op: (producer op,
covered buffers)}): a launch that waits on the device for a producer launch on another
stream to publish its part (the persistent backward's bucket counters: engine.py
`_emit_persist_overlap`, the one-wave `prn_bucket_wait` kernel).  A bare producer index
orders everything after the wait on its stream after the WHOLE producer.  With a set of
covered buffer names the ordering is partial -- the producer still runs and still uses
other buffers: until that stream is ordered after the producer by an event, every launch
after the wait must declare the buffers it reads or writes (`op_buffers` {op: names}) and
touch only buffers some earlier wait on its stream covered (R5); a collective among them
satisfies R4 against the producer only through that coverage.  What a count covers (the
bucket's gradients, slabs and parameters, which the producer publishes complete and no
longer reads after the count) is the engine's claim; this check holds the comm stream's
ops to it (a misassigned bucket or a weight the backward still reads is caught).

Op encoding (`Plan.op_kinds` / `op_streams` / `op_events`): kind 0 launch,
1 record, 2 wait, 3 timing probe (ignored); stream 0 main, 1 side, 2 comm.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Sequence, Tuple

LAUNCH, RECORD, WAIT, TIMING = 0, 1, 2, 3
NSTREAMS = 3
_COLLECTIVES = ("all_reduce",)


def check_plan_order(kinds: Sequence[int], streams: Sequence[int], events: Sequence[int],
                     segments: Iterable[Tuple[str, int, int]],
                     names: Sequence[str] | None = None,
                     barriers: Sequence[int] = (),
                     device_deps: Dict[int, object] | None = None,
                     op_buffers: Dict[int, Iterable[str]] | None = None) -> List[str]:
    """Return a list of human-readable violations (empty = ordering is sound).

    ``barriers``: plan indices where the host runs a collective on the main
    stream between two Plan.run calls (the op at that index has not been issued
    yet); checked with rule R4 like an all-reduce op at that position."""
    n = len(kinds)
    if len(streams) != n or len(events) != n:
        raise ValueError("kinds/streams/events length mismatch")
    errs: List[str] = []
    barrier_set = set(barriers)

    def op(i: int) -> str:
        return f"op {i}" + (f" ({names[i]})" if names is not None and i < n else "")

    for seg, a, b in segments:
        if not (0 <= a <= b <= n):
            errs.append(f"{seg}: bad range [{a}, {b}) for a plan of {n} ops")
            continue
        # clock[s][t]: latest plan index of a launch on stream t known to complete
        # before the current point of stream s (-1: none); launched[t]: latest
        # launch on t so far.  fork[s]: stream s is ordered after a main record.
        clock = [[-1] * NSTREAMS for _ in range(NSTREAMS)]
        rec: Dict[int, Tuple[int, List[int], bool]] = {}   # event -> (stream, clock, forked)
        forked = [True, False, False]
        launched = [-1] * NSTREAMS
        reported_fork = [False] * NSTREAMS
        # partial[s]: (producer op, buffers covered so far) of the device waits on stream s
        # whose producer stream s is not yet ordered after
        partial: Dict[int, Tuple[int, set]] = {}

        def bufs(i: int):
            got = (op_buffers or {}).get(i)
            return None if got is None else set(got)

        def r4(i: int, s: int, what: str):
            for t in range(NSTREAMS):
                if t != s and launched[t] > clock[s][t]:
                    p = partial.get(s)
                    b = bufs(i)
                    if (p is not None and launched[t] == p[0] and b is not None
                            and b <= p[1]):
                        continue   # ordered after the producer's covered part (R5)
                    errs.append(f"{seg}: {what} at {op(i)} is not ordered after {op(launched[t])} "
                                f"on stream {t} (R4)")

        for i in range(a, b):
            if i in barrier_set:
                r4(i, 0, "host all-reduce split")
            k, s, e = kinds[i], streams[i], events[i]
            if not 0 <= s < NSTREAMS:
                errs.append(f"{seg}: {op(i)} on unknown stream {s}")
                continue
            if k == RECORD:
                rec[e] = (s, list(clock[s]), forked[s])
            elif k == WAIT:
                src = rec.get(e)
                if src is None:
                    errs.append(f"{seg}: {op(i)} waits on event {e} not recorded earlier "
                                f"in the segment (R1)")
                    continue
                if src[0] == s:
                    errs.append(f"{seg}: {op(i)} waits on event {e} recorded on its own "
                                f"stream (R1: no cross-stream ordering)")
                    continue
                clock[s] = [max(x, y) for x, y in zip(clock[s], src[1])]
                forked[s] = forked[s] or src[2]
            elif k == LAUNCH:
                dep = (device_deps or {}).get(i)
                covered = None
                if isinstance(dep, tuple):
                    dep, covered = dep[0], set(dep[1])
                p = partial.get(s)
                if p is not None and clock[s][streams[p[0]]] >= p[0]:
                    partial.pop(s)   # an event has since ordered s after the whole producer
                    p = None
                if dep is not None:
                    if not (a <= dep < i) or kinds[dep] != LAUNCH or streams[dep] == s:
                        errs.append(f"{seg}: device dependency of {op(i)} on {op(dep)} is not "
                                    f"an earlier launch of this segment on another stream")
                    elif covered is None:
                        t = streams[dep]
                        clock[s][t] = max(clock[s][t], dep)
                    elif p is not None and p[0] != dep:
                        errs.append(f"{seg}: {op(i)} adds a partial device dependency on "
                                    f"{op(dep)} beside one on {op(p[0])} (R5)")
                    else:
                        partial[s] = (dep, (p[1] if p is not None else set()) | covered)
                        p = partial[s]
                elif p is not None:
                    b = bufs(i)
                    if b is None:
                        errs.append(f"{seg}: {op(i)} runs beside {op(p[0])} (a partial device "
                                    f"dependency) without declaring its buffers (R5)")
                    elif not b <= p[1]:
                        errs.append(f"{seg}: {op(i)} touches {sorted(b - p[1])} while "
                                    f"{op(p[0])} may still use them: only {sorted(p[1])} are "
                                    f"covered by the device waits before it (R5)")
                if s != 0 and not forked[s] and not reported_fork[s]:
                    errs.append(f"{seg}: stream-{s} {op(i)} before any fork from the main "
                                f"stream (R2)")
                    reported_fork[s] = True
                if names is not None and names[i] in _COLLECTIVES:
                    r4(i, s, names[i])
                clock[s][s] = i
                launched[s] = i
        if b in barrier_set:
            r4(b, 0, "host all-reduce split")
        for t in (1, 2):
            if launched[t] > clock[0][t]:
                errs.append(f"{seg}: stream-{t} work up to {op(launched[t])} is never "
                            f"joined into the main stream before the segment ends (R3)")
    return errs


def check_plan(plan, segments: Dict[str, Tuple[int, int]], barriers: Sequence[int] = (),
               device_deps: Dict[int, object] | None = None,
               op_buffers: Dict[int, Iterable[str]] | None = None) -> List[str]:
    """`check_plan_order` over a native `_C.Plan` and the engine's {name: (a, b)}."""
    return check_plan_order(plan.op_kinds(), plan.op_streams(), plan.op_events(),
                            [(k, a, b) for k, (a, b) in segments.items()], plan.names(),
                            barriers=barriers, device_deps=device_deps, op_buffers=op_buffers)
