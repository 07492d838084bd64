"""Host-side stream-ordering check of a recorded native Plan (race detection).

The training step is a static list of ops on two HIP streams (main = 0, side = 1)
ordered only by event record/wait pairs (engine.py `_flush_side` / `_flush_buckets`).
A missing fork or join is a data race that no GPU sanitizer on this pool can find
(no XNACK / GPU ASan), and it usually shows up only as rare, non-reproducible
gradient corruption.  This module checks the op list statically, once, when the
engine builds the plan (SURVEY.md §5 "Race detection": stream-ordering asserts
around comm/compute events; the reference has none -- its only checks are graph
asserts, `/root/reference/vgg_preprocessing.py:67-84`, `cifar_input.py:110-115`).

Rules, per segment (a range of ops the host runs with one `Plan.run` call):

R1  every wait names an event recorded earlier in the same segment, on the other
    stream (a wait on a never-recorded event is a no-op: no ordering at all; a
    record from a previous segment may be a previous step's);
R2  fork: every side-stream launch follows a side-stream wait on an event the main
    stream recorded in the same segment (otherwise it races with the work the host
    queued before the segment, e.g. the previous step's optimizer);
R3  join: if the segment launched anything on the side stream, the main stream
    waits, before the segment ends, on an event the side stream recorded after its
    last launch (otherwise the next segment / all-reduce / optimizer reads
    gradients that are still being written).

Op encoding (`Plan.op_kinds` / `op_streams` / `op_events`): kind 0 launch,
1 record, 2 wait; stream 0 main, 1 side.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Sequence, Tuple

LAUNCH, RECORD, WAIT = 0, 1, 2


def check_plan_order(kinds: Sequence[int], streams: Sequence[int], events: Sequence[int],
                     segments: Iterable[Tuple[str, int, int]],
                     names: Sequence[str] | None = None) -> List[str]:
    """Return a list of human-readable violations (empty = ordering is sound)."""
    n = len(kinds)
    if len(streams) != n or len(events) != n:
        raise ValueError("kinds/streams/events length mismatch")
    errs: List[str] = []

    def op(i: int) -> str:
        return f"op {i}" + (f" ({names[i]})" if names is not None else "")

    for seg, a, b in segments:
        if not (0 <= a <= b <= n):
            errs.append(f"{seg}: bad range [{a}, {b}) for a plan of {n} ops")
            continue
        rec: Dict[int, Tuple[int, int]] = {}   # event -> (stream, index) of latest record
        forked = False                         # side stream ordered after main in this segment
        last_side_launch = -1
        joined_after = -1                      # latest side index a main wait has joined
        for i in range(a, b):
            k, s, e = kinds[i], streams[i], events[i]
            if k == RECORD:
                rec[e] = (s, i)
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
                if s == 1:
                    forked = True
                else:
                    joined_after = max(joined_after, src[1])
            elif k == LAUNCH and s == 1:
                if not forked:
                    errs.append(f"{seg}: side-stream {op(i)} before any fork from the main "
                                f"stream (R2)")
                    forked = True   # report once per segment
                last_side_launch = i
        if last_side_launch >= 0 and joined_after < last_side_launch:
            errs.append(f"{seg}: side-stream work up to {op(last_side_launch)} is never "
                        f"joined into the main stream before the segment ends (R3)")
    return errs


def check_plan(plan, segments: Dict[str, Tuple[int, int]]) -> List[str]:
    """`check_plan_order` over a native `_C.Plan` and the engine's {name: (a, b)}."""
    return check_plan_order(plan.op_kinds(), plan.op_streams(), plan.op_events(),
                            [(k, a, b) for k, (a, b) in segments.items()], plan.names())
