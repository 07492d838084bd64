"""Gradient bucketing for the data-parallel all-reduce.

Trainables live in one flat fp32 buffer in TF creation order, and backward
produces their gradients roughly in reverse creation order.  A bucket is
therefore just a contiguous slice ``[lo, hi)`` of that buffer, built from the
end: no packing copies, one RCCL all-reduce per bucket, issued as soon as the
backward op that finalises the bucket's last gradient has been enqueued.

Replaces Horovod's runtime tensor-fusion buffer ("Horovod C++
core"): the ResNet graph is static, so the fusion plan is computed once.
Bucket size trades latency (fewer, larger collectives over the point-to-point
xGMI ring: 2(n-1) latency hops each) against overlap (the last bucket cannot
start before backward ends).
"""
from __future__ import annotations


def assign_buckets(slots, bucket_bytes: int, elem_bytes: int = 4):
    """slots: objects with .offset/.numel in creation order.  Returns a list of
    (lo, hi, [slot names]) ordered from the END of the buffer (= backward order)."""
    buckets = []
    cur = []
    cur_bytes = 0
    for s in reversed(slots):
        cur.append(s)
        cur_bytes += s.numel * elem_bytes
        if cur_bytes >= bucket_bytes:
            buckets.append(cur)
            cur, cur_bytes = [], 0
    if cur:
        buckets.append(cur)
    out = []
    for b in buckets:
        lo = min(s.offset for s in b)
        hi = max(s.offset + s.numel for s in b)
        out.append((lo, hi, [s.name for s in b]))
    # contiguity sanity: buckets tile the buffer exactly
    spans = sorted((lo, hi) for lo, hi, _ in out)
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 == b0, "buckets must tile the flat buffer"
    return out


def schedule_buckets(buckets, ready_index: dict):
    """Attach to each bucket the plan index after which all its gradients are
    final; returns [(ready_idx, lo, hi)] sorted by ready_idx (stable)."""
    sched = []
    for lo, hi, names in buckets:
        idx = max(ready_index[n] for n in names)
        sched.append((idx, lo, hi))
    sched.sort(key=lambda t: t[0])
    return sched
