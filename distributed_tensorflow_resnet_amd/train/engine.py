"""GPU training engine: flat buffers + one static native plan per step.

This replaces the reference's TF graph + MonitoredTrainingSession hot loop
(`mon_sess.run(train_op)`, resnet_cifar_main.py:339-358).  The
ResNet v2 graph is static, so instead of an autograd tape the engine records
ONE native plan (csrc/bindings.cpp `Plan`) holding every launch of a training
step with all pointers bound:

  forward   input augmentation -> stem -> blocks -> BN-ReLU+avg-pool -> dense ->
            softmax-xent (+training precision, +dense-bias grad)
            * BN-ReLU is never materialised: each conv applies the previous BN's
              scale/shift + ReLU while staging its A operand (PRE), and emits the
              next BN's Welford partials from its epilogue (STATS);
            * the residual add is fused into the last conv of each block;
  backward  hand-scheduled reverse pass: per conv a dgrad (MFMA) and a split-K
            wgrad (MFMA, fused BN-ReLU recompute of its input) + deterministic
            reduce into the flat fp32 gradient; per BN one reduce / finalize /
            apply (ReLU mask and residual-gradient add fused);
  allreduce after the op that finalises each gradient bucket
            (parallel/buckets.py): a plan op on the comm stream -- the native
            RCCL communicator (csrc/comm.h) all-reduces the bucket while the
            compute streams continue the backward; the optimizer waits on it
            (c10d all-reduces between plan segments for gloo rehearsals);
  optimizer one fused SGD-momentum + weight-decay + bf16 re-pack launch, LR from
            the device-resident global_step, then global_step += 1.

The plan runs natively segment by segment (no Python per op); `use_graph`
captures the whole step into a hipGraph instead (measured slower than the eager
native plan on this runtime, profiles/launch_mode_ab.md).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import native
from ..models.params import ParamStore
from ..models.spec import BNSpec, ConvSpec, ModelSpec
from ..parallel.buckets import assign_buckets, schedule_buckets
from ..utils import tune
from ..utils.streamcheck import check_plan

BF16 = torch.bfloat16
BN_DECAY = 0.997
# Diagnostics: DTR_DIAG_SKIP=wgrad,dgrad,... drops those launches (wrong math; timing only)
_DIAG_SKIP = set(filter(None, os.environ.get("DTR_DIAG_SKIP", "").split(",")))
from ..ops.reference import BN_EPS  # noqa: E402  (TF's effective 1.001e-5)

WGD_DTYPE = np.dtype([
    ("part", "<u8"), ("grad", "<u8"), ("splits", "<i4"), ("K", "<i4"), ("Kv", "<i4"),
    ("taps", "<i4"), ("C", "<i4"), ("Cv", "<i4"), ("chunk0", "<i8"),
])

SEG_DTYPE = np.dtype([
    ("offset", "<i8"), ("numel", "<i8"), ("bf_ohwi", "<i8"), ("bf_hwio", "<i8"),
    ("kh", "<i4"), ("kw", "<i4"), ("C", "<i4"), ("K", "<i4"), ("cpad", "<i4"), ("kpad", "<i4"),
])

OPTW_DTYPE = np.dtype([   # csrc/optim.h OptWork
    ("part", "<u8"), ("tile0", "<i8"), ("splits", "<i4"), ("kslab", "<i4"), ("cslab", "<i4"),
    ("tiled", "<i4"), ("tr", "<i4"), ("tc", "<i4"),
])

OPT_TILE_LOADS = 2048   # a sgd_tiles workgroup's slab loads: <= 8 16-byte loads per thread


class PersistentStepError(RuntimeError):
    """A persistent CIFAR launch's grid barrier timed out (csrc/cifar_persist.hip: every
    wait is bounded, a timed-out workgroup sets the error flag and exits).  The step's
    results are invalid; the driver exits with code 3 so parallel/launch.py restarts the
    job from the last good checkpoint, on the per-layer plan."""


def _pow2ceil(x: int) -> int:
    return 1 << max(0, (int(x) - 1).bit_length())


def opt_tile(R: int, K: int, splits: int, cslab: int, C: int, taps: int, nosplit=(64, 64)):
    """Tile (rows tap*C+ci, output channels) of a weight in the one-launch optimizer
    (csrc/optim.hip sgd_tiles_kernel): 64 x 64 without slabs; with `splits` slabs the
    tile shrinks (columns first) until its float4 slab loads fit OPT_TILE_LOADS and,
    past 8 splits (4 thread groups of 64 float4 units), until it has <= 64 units.
    Padded slab rows (cslab != C, the stem) keep all rows in one tile."""
    if splits == 0:
        return nosplit
    units_max = 64 if splits > 8 else 1 << 30
    TC = min(64, _pow2ceil(K))
    if cslab != C:
        assert R <= 64 and (taps * cslab) % 4 == 0, (R, taps, cslab)
        cols4 = taps * cslab // 4
        while TC > 1 and (TC * cols4 * splits > OPT_TILE_LOADS or TC * cols4 > units_max):
            TC //= 2
        assert TC * cols4 <= units_max, (R, K, splits, cslab)
        return R, TC
    assert C % 4 == 0, C
    TR = min(64, _pow2ceil(R))
    while (TR * TC // 4) * splits > OPT_TILE_LOADS or TR * TC // 4 > units_max:
        if TC >= TR and TC > 1:
            TC //= 2
        elif TR > 4:
            TR //= 2
        else:
            break
    assert TR * TC // 4 <= units_max, (R, K, splits)
    return TR, TC


@dataclass
class LRSchedule:
    """Piecewise LR evaluated on the device (see csrc/optim.h LrSchedule)."""
    init: float
    bounds: list
    values: list
    warm_steps: int = 0
    warm_from: float = 0.0
    warm_to: float = 0.0

    def at(self, step: int) -> float:
        """Host mirror of the device formula (used by hooks/tests)."""
        if step <= 0:
            return self.init
        t = step - 1
        if t < self.warm_steps:
            return self.warm_from + (self.warm_to - self.warm_from) * t / self.warm_steps
        for b, v in zip(self.bounds, self.values):
            if t < b:
                return v
        return self.values[-1]


def cifar_lr_schedule() -> LRSchedule:
    """resnet_cifar_main.py:304-324 (begin() = 0.1)."""
    return LRSchedule(0.1, [40000, 60000, 80000], [0.1, 0.01, 0.001, 0.0001])


def imagenet_lr_schedule() -> LRSchedule:
    """resnet_imagenet_main.py:306-329: warm-up 0.1->0.4 over 6240 steps (begin()=0.4)."""
    return LRSchedule(0.4, [37440, 74880, 99840], [0.4, 0.04, 0.004, 0.0004],
                      warm_steps=6240, warm_from=0.1, warm_to=0.4)


def scaled(s: LRSchedule, factor: float) -> LRSchedule:
    """The same schedule with its step boundaries (and warm-up length) x factor."""
    if factor == 1.0:
        return s
    return LRSchedule(s.init, [max(1, int(round(b * factor))) for b in s.bounds], list(s.values),
                      int(round(s.warm_steps * factor)), s.warm_from, s.warm_to)


def lr_values_scaled(s: LRSchedule, factor: float) -> LRSchedule:
    """The same schedule with every LR value (and the warm-up's ends) x factor."""
    if factor == 1.0:
        return s
    return LRSchedule(s.init * factor, list(s.bounds), [v * factor for v in s.values],
                      s.warm_steps, s.warm_from * factor, s.warm_to * factor)


def constant_lr(lr: float) -> LRSchedule:
    return LRSchedule(lr, [], [lr])


# partial count meaning "the pointer is a fp64 accumulator" in the pointer-vector
# arguments of plan.conv_gemm (pfin / abwd; read back as int -1 by the bindings)
_ACC_CNT = 0xFFFFFFFF


def _ceil(a, b):
    return (a + b - 1) // b


@dataclass
class _BN:
    spec: BNSpec
    gamma: int          # pointers into master / grad / stats buffers
    beta: int
    dgamma: int
    dbeta: int
    mmean: int
    mvar: int
    mean: torch.Tensor = None
    rstd: torch.Tensor = None
    scale: torch.Tensor = None
    shift: torch.Tensor = None
    # forward statistics not yet finalized: (partials ptr, count, rows per partial, M)
    pending: tuple = None
    names: tuple = ()
    part: torch.Tensor = None     # this BN's forward tile partials [T][2][C]
    bpart: torch.Tensor = None    # backward partial sums [T][2][C]
    acc: torch.Tensor = None      # accumulator mode: fp64 [REP][2][C] sum y, sum y^2
    bacc: torch.Tensor = None     # ... and sum g, sum g*xhat (zeroed once per step)


@dataclass
class _Conv:
    spec: ConvSpec
    cin: int            # effective (padded) input channels
    ohwi: int           # bf16 pointers
    hwio: int
    grad: int           # fp32 gradient pointer (TF HWIO)
    cin_valid: int
    name: str = ""


class Engine:
    """Owns all device state of one data-parallel rank."""

    def __init__(self, spec: ModelSpec, batch_size: int, *, weight_decay: float,
                 lr_schedule: LRSchedule, optimizer: str = "mom", momentum: float = 0.9,
                 device=None, dist_ctx=None, bucket_mb: float | None = None, reduce_mb: float | None = None,
                 seed: int = 0,
                 input_mode: str = "auto", global_batch: int | None = None,
                 use_graph: bool = False, data_seed: int = 1234, fork_wgrad: bool | None = None,
                 allreduce_dtype: str = "fp32", native_comm: bool | None = None, comm=None):
        self.nat = native(required=True)
        tune.validate(k for k, *_ in self.nat.tune_table())
        self.spec = spec
        self.N = batch_size
        self.device = torch.device(device or "cuda")
        self.dist = dist_ctx
        self.world = dist_ctx.world_size if dist_ctx is not None else 1
        self.global_batch = global_batch or batch_size * self.world
        self.wd = float(weight_decay)
        self.momentum = float(momentum)
        self.use_momentum = optimizer == "mom"
        self.sched = lr_schedule
        self.use_graph = use_graph
        self.data_seed = data_seed
        if allreduce_dtype not in ("fp32", "bf16"):
            raise ValueError(f"allreduce_dtype must be fp32 or bf16, got {allreduce_dtype!r}")
        # bf16 gradient exchange: each bucket is cast into a bf16 staging buffer, all-reduced
        # (half the xGMI bytes) and cast back into the fp32 flat gradient before the update
        self.allreduce_bf16 = allreduce_dtype == "bf16"
        if fork_wgrad is None:
            # measured: eager + forked wgrad stream beats hipGraph replay (which
            # handles the cross-stream event edges poorly); graphs stay single-stream
            fw = tune.get("fork_wgrad")
            fork_wgrad = (not use_graph) if fw < 0 else bool(fw)
        # residual blocks per side-stream fork (tune fork_every)
        fe = tune.get("fork_every")
        self.fork_every = max(1, fe if fe > 0 else (4 if spec.dataset.startswith("cifar") else 2))
        # Backward tail: the weight gradients still queued for the side stream when the
        # main stream's dgrad chain ends (the first stage's) are shared out -- this
        # fraction of them, the last-queued ones, runs on the otherwise idle main stream
        # after the stem (_split_tail).  0 = all on the side stream.  Measured (CIFAR RN50,
        # ms/step, 0 / 0.5 / 0.75 / 1): bs16 0.978 / 0.972 / 0.972 / 0.970, bs32 1.002 /
        # 0.994 / 1.017 / 1.011, bs64 1.128 / 1.131 / 1.131 / 1.130, bs128 1.326 / 1.316 /
        # 1.314 / 1.303 (scripts/ab_tail.sh).  ImageNet, after the streaming 1x1 kernels
        # shortened the main stream's chain: RN50 bs128 1 / 0.5 / 0.25 = 10.56 / 10.49 /
        # 10.49 ms, RN101 bs256 1 / 0.5 = 32.78 / 32.66 ms (scripts/gpurun/gpu_r3_final.sh).
        tm = tune.get("tail_main")
        if tm < 0:
            tm = 1.0 if spec.dataset.startswith("cifar") else 0.5
        self.tail_main = min(1.0, max(0.0, tm))
        # ...and the last reduces then run on the main stream behind one join
        # (reduce_main_tail=0: forked to the side stream like the earlier buckets)
        self.reduce_main_tail = bool(tune.get("reduce_main_tail"))
        self.markers = os.environ.get("DTR_ROCTX", "0") != "0"
        self.fork_wgrad = fork_wgrad
        if input_mode == "auto":
            input_mode = "cifar_u8" if spec.dataset.startswith("cifar") else "nhwc"
        self.input_mode = input_mode
        self.kpad = _ceil(spec.num_classes, 16) * 16
        self.cpad_in = 8
        # ImageNet stem as a space-to-depth 4x4/1 conv over [N, H/2, W/2, 16] (data.hip
        # stem_s2d_*: K 392 -> 256, stride-1 gathers, a 2-tile weight gradient instead of 4)
        st = spec.stem
        self.stem_s2d = (bool(tune.get("stem_s2d")) and st.kh == 7 and
                         st.kw == 7 and st.stride == 2 and st.cin <= 3 and
                         spec.image_h % 2 == 0 and spec.image_w % 2 == 0 and
                         2 * st.ho == spec.image_h and 2 * st.wo == spec.image_w)

        dev = self.device
        self.params = ParamStore(spec, device=dev)
        self.params.initialize(seed)
        self.grad = torch.zeros(self.params.n_train, device=dev)
        self.mom = torch.zeros(self.params.n_train, device=dev)
        self.gstep = torch.zeros(1, dtype=torch.int64, device=dev)
        self.scalars = torch.zeros(8, device=dev)  # loss_sum, correct, lr, l2
        # weight-gradient and all-reduce streams: one pair per process, created before
        # the process group's (parallel/dist.py engine_streams: hardware queue order)
        from ..parallel.dist import engine_streams
        self.side, self.comm_stream = engine_streams(dev)
        # Native communicator (csrc/comm.h: RCCL, or the shm rehearsal transport):
        # the bucket all-reduces are plan ops on the comm stream.  None: world 1
        # (nothing to reduce), the c10d transport, or a fallback after a failed
        # native init (c10d all-reduces issued by the host between plan segments,
        # _run_bwd; the reason in comm_fallback_reason).  native_comm=True forces
        # a single-rank RCCL communicator, `comm=` takes a prebuilt one (tests:
        # _C.Comm.loopback(2), the doubling stand-in for an all-reduce).
        self.comm = comm
        self.comm_fallback_reason = None
        didx = dev.index if dev.index is not None else torch.cuda.current_device()
        if comm is not None:
            pass
        elif self.dist is not None and (self.world > 1 or native_comm):
            if native_comm is not False:
                self.comm = self.dist.native_comm(didx, force=bool(native_comm))
                self.comm_fallback_reason = self.dist.comm_fallback_reason
        elif native_comm:
            from ..parallel.dist import DistContext
            self.comm = DistContext().native_comm(didx, force=True)
        self.grad_bf16 = (torch.zeros(self.params.n_train, dtype=BF16, device=dev)
                          if self.allreduce_bf16 and (self.world > 1 or self.comm is not None)
                          else None)
        self._build_weight_layout()
        self._alloc_activations()
        # Persistent small-batch CIFAR step (train/persist.py, csrc/cifar_persist.hip): the
        # forward and the backward each as ONE launch (tune persist: -1 auto = per-rank
        # batch <= AUTO_MAX_BATCH on a supported CIFAR network, 0 off, 1 whenever supported)
        from . import persist as _persist
        from ..parallel.dist import gpu_shared_by_ranks
        pm = tune.get("persist")
        self.persist_slices = tune.get("persist_slices")
        self.persist_overlap_tune = bool(tune.get("persist_overlap"))
        self.opt_fused = bool(tune.get("opt_fused"))
        # why the persistent step is off ("" = on); never on a GPU shared by several ranks
        # (its grids need every CU to themselves), and the same choice on EVERY rank (the
        # two plans issue different collectives)
        if pm == 0:
            reason = "tune persist=0"
        elif pm != 1 and self.N > _persist.AUTO_MAX_BATCH:
            reason = f"per-rank batch {self.N} > {_persist.AUTO_MAX_BATCH} (auto)"
        elif gpu_shared_by_ranks(self.dist, didx):
            reason = "GPU shared by several ranks"
        else:
            reason = _persist.check(self)
        if self.dist is not None and self.dist.active and not self.dist._agree(reason == ""):
            reason = reason or "another rank cannot run the persistent step"
        self.persist_reason = reason
        self.persist = reason == ""
        # world > 1 (or a forced communicator): the gradient buckets' reduces and
        # all-reduces overlap the persistent backward launch (tune persist_overlap)
        self.persist_overlap = self.persist and _persist.overlap_planned(self)
        if self.persist and self.dist is not None and self.dist.active:
            # one plan shape on every rank (3 bucket all-reduces or 1)
            self.persist_overlap = self.dist._agree(self.persist_overlap)
        self.prn = _persist.PersistStep(self) if self.persist else None
        self.plan = self.nat.Plan()
        self._keep = []   # tensors referenced by the plan
        self.ready_index: dict[str, int] = {}
        # stream check: device-side waits (op -> producer op, or (producer op, buffers the
        # wait covers)) and the buffers the ops running beside a partial wait touch
        self._device_deps: dict = {}
        self._op_buffers: dict[int, set] = {}
        self.reduce_buckets = self.world > 1 or self.comm is not None
        if self.reduce_buckets:
            if not bucket_mb:
                # ~4 buckets, at most 25 MB each: ImageNet RN50's 97 MB of gradients in
                # 25 MB all-reduces overlapping the backward; CIFAR RN50's 2.9 MB in four,
                # so all but the last (stage 1's small kernels) overlap the backward
                # instead of one latency-bound all-reduce after it
                bucket_mb = min(25.0, 4.0 * self.params.n_train / 2 ** 20 / 4)
            self.buckets = assign_buckets(self.params.train_slots, int(bucket_mb * 2 ** 20))
        else:  # one bucket: nothing to all-reduce, only the split-K reduces
            self.buckets = [(0, self.params.n_train, [s.name for s in self.params.train_slots])]
        # Split-K reduce groups nest inside the buckets: each group's grouped reduce
        # runs on the side stream as soon as its weight gradients are queued, so
        # only the last group's reduce (stem + first stage) sits at the end of
        # backward.  (One reduce of all of ResNet-50's slabs at the end was ~0.45 ms
        # of tail; the group size trades that tail against launch count.)
        if reduce_mb is None:
            # ~6 groups, at most 4 MB each (measured: CIFAR RN50's 3 MB of gradients in
            # 0.5 MB groups -2.3 % step time vs one group, whose 78 us reduce of 290 MB
            # of split-K slabs sat alone at the end of backward)
            reduce_mb = min(4.0, 4.0 * self.params.n_train / 2 ** 20 / 6)
        if tune.get("reduce_mb") > 0:
            reduce_mb = tune.get("reduce_mb")
        slot_of = {s.name: s for s in self.params.train_slots}
        self.reduce_groups = []
        for lo, hi, names in self.buckets:
            sub = assign_buckets([slot_of[n] for n in names], int(reduce_mb * 2 ** 20))
            self.reduce_groups.append([g[2] for g in sub])
        self._build_train_plan()
        if self.reduce_buckets and self.comm is None:
            # gloo rehearsal: the host issues each bucket's c10d all-reduce at its
            # ready index, between Plan.run calls (_run_bwd)
            self.bucket_sched = schedule_buckets(self.buckets, self.ready_index)
        else:
            self.bucket_sched = []
        errs = check_plan(self.plan, self.seg, barriers=[i for i, _, _ in self.bucket_sched],
                          device_deps=self._device_deps, op_buffers=self._op_buffers)
        if errs:   # fork/join structure of the three streams (race check)
            raise RuntimeError("plan stream-ordering violations:\n  " + "\n  ".join(errs[:8]))
        self.graph = None
        self._captured = False
        self._steps_run, self._cost_at = 0, -1
        self.eval_plans = {}
        self.repack()

    # ------------------------------------------------------------------ layout
    def _build_weight_layout(self):
        spec = self.spec
        ps = self.params
        mptr = ps.master.data_ptr()
        gptr = self.grad.data_ptr()
        segs = []
        bf_total = 0
        self.convs: dict[str, _Conv] = {}
        conv_specs = {c.name: c for c in spec.all_convs()}
        for s in ps.train_slots:
            rec = np.zeros(1, dtype=SEG_DTYPE)[0]
            rec["offset"], rec["numel"] = s.offset, s.numel
            rec["bf_ohwi"] = rec["bf_hwio"] = -1
            if s.kind == "conv":
                c = conv_specs[s.name.split("/")[0]]
                taps = c.kh * c.kw
                cpad = self.cpad_in if c.cin < 8 else c.cin
                rec["kh"], rec["kw"], rec["C"], rec["K"] = c.kh, c.kw, c.cin, c.cout
                rec["cpad"], rec["kpad"] = cpad, c.cout
                if self.stem_s2d and c.name == spec.stem.name:
                    rec["bf_ohwi"] = -1   # its OHWI operand comes from stem_s2d_pack
                else:
                    rec["bf_ohwi"] = bf_total
                    bf_total += c.cout * taps * cpad
                if c.cin >= 8:   # the stem never needs dgrad
                    rec["bf_hwio"] = bf_total
                    bf_total += taps * c.cin * c.cout
            elif s.kind == "dense_kernel":
                F, classes = s.shape
                rec["kh"], rec["kw"], rec["C"], rec["K"] = 1, 1, F, classes
                rec["cpad"], rec["kpad"] = F, self.kpad
                rec["bf_ohwi"] = bf_total
                bf_total += self.kpad * F
                rec["bf_hwio"] = bf_total
                bf_total += F * self.kpad
            else:
                rec["kh"] = rec["kw"] = 1
                rec["C"], rec["K"] = 1, 1
                rec["cpad"], rec["kpad"] = 1, 1
            segs.append(rec)
        seg_arr = np.array(segs, dtype=SEG_DTYPE)
        assert SEG_DTYPE.itemsize == self.nat.param_seg_bytes()
        self.seg_arr, self.seg_names = seg_arr, [s.name for s in ps.train_slots]
        self.segs = torch.from_numpy(seg_arr.view(np.uint8).copy()).to(self.device)
        self.nseg = len(segs)
        # OHWI transpose tiles (ohwi_pack): ceil(taps*C/64) x ceil(K/64) per weight
        tiles = [(_ceil(int(r["kh"] * r["kw"] * r["C"]), 64) * _ceil(int(r["K"]), 64)
                  if r["bf_ohwi"] >= 0 else 0) for r in seg_arr]
        self.ohwi_tiles = int(sum(tiles))
        self.ohwi_tile0 = torch.tensor(np.concatenate([[0], np.cumsum(tiles)[:-1]]).astype(np.int64),
                                       device=self.device)
        self.wbf = torch.zeros(max(bf_total, 1), dtype=BF16, device=self.device)
        bptr = self.wbf.data_ptr()
        for rec, s in zip(seg_arr, ps.train_slots):
            if s.kind == "conv":
                c = conv_specs[s.name.split("/")[0]]
                cin = self.cpad_in if c.cin < 8 else c.cin
                ohwi = bptr + 2 * int(rec["bf_ohwi"])
                if self.stem_s2d and c.name == spec.stem.name:
                    cin = 16
                    self.stem_w4 = torch.zeros(c.cout * 256, dtype=BF16, device=self.device)
                    self.stem_g4 = torch.zeros(c.cout * 256, device=self.device)
                    self.stem_master = mptr + 4 * s.offset
                    ohwi = self.stem_w4.data_ptr()
                self.convs[c.name] = _Conv(
                    c, cin, ohwi,
                    bptr + 2 * int(rec["bf_hwio"]) if rec["bf_hwio"] >= 0 else 0,
                    gptr + 4 * s.offset, c.cin, s.name)
            elif s.kind == "dense_kernel":
                self.dense_ohwi = bptr + 2 * int(rec["bf_ohwi"])
                self.dense_hwio = bptr + 2 * int(rec["bf_hwio"])
                self.dense_grad = gptr + 4 * s.offset
                self.dense_name = s.name
        bslot = ps.slot("dense/bias")
        self.dense_bias = mptr + 4 * bslot.offset
        self.dense_bias_grad = gptr + 4 * bslot.offset

        # BatchNorm bookkeeping
        self.bns: dict[str, _BN] = {}
        sptr = ps.stats.data_ptr()
        bn_specs = [b for blk in spec.blocks for b in blk.bns] + [spec.final_bn]
        total_c = sum(b.channels for b in bn_specs)
        self.bnbuf = torch.zeros(4 * total_c, device=self.device)
        # last-arriver counters for the in-kernel BN finalize (bump-allocated per fused
        # launch at plan build; the kernels leave them zeroed) + group-partial scratch
        off = 0
        for b in bn_specs:
            g = ps.slot(f"{b.name}/gamma")
            be = ps.slot(f"{b.name}/beta")
            mm = ps.slot(f"{b.name}/moving_mean")
            mv = ps.slot(f"{b.name}/moving_variance")
            C = b.channels
            e = _BN(b, mptr + 4 * g.offset, mptr + 4 * be.offset, gptr + 4 * g.offset,
                    gptr + 4 * be.offset, sptr + 4 * mm.offset, sptr + 4 * mv.offset,
                    names=(g.name, be.name))
            e.mean = self.bnbuf[off:off + C]
            e.rstd = self.bnbuf[total_c + off:total_c + off + C]
            e.scale = self.bnbuf[2 * total_c + off:2 * total_c + off + C]
            e.shift = self.bnbuf[3 * total_c + off:3 * total_c + off + C]
            off += C
            self.bns[b.name] = e

    def _alloc_activations(self):
        spec, N, dev = self.spec, self.N, self.device
        H, W = spec.image_h, spec.image_w
        if self.input_mode == "cifar_u8":
            self.img_u8 = torch.zeros((N, 3, H, W), dtype=torch.uint8, device=dev)
        elif self.input_mode == "imagenet_u8":   # VGG crops, HWC (imagenet_u8_pack)
            self.img_u8 = torch.zeros((N, H, W, 3), dtype=torch.uint8, device=dev)
        self.x_in = torch.zeros(self._x_in_shape(N), dtype=BF16, device=dev)
        self.labels = torch.zeros(N, dtype=torch.int32, device=dev)
        st = spec.stem
        self.stem_out = torch.empty((N, st.ho, st.wo, st.cout), dtype=BF16, device=dev)
        if spec.maxpool:
            mh = _ceil(st.ho, 2)
            self.pool_out = torch.empty((N, mh, mh, st.cout), dtype=BF16, device=dev)
            self.pool_arg = torch.empty((N, mh, mh, st.cout), dtype=torch.uint8, device=dev)
        self.X = []     # block inputs (X[i] = input of block i, X[-1] = last output)
        self.H1, self.H2 = [], []
        x0 = self.pool_out if spec.maxpool else self.stem_out
        self.X.append(x0)
        max_act = x0.numel()
        sc_max = 0
        self.Y1, self.Y2 = [], []   # materialized inner BN-ReLU outputs (_materialize_bn)
        for b in spec.blocks:
            f = b.convs[0].cout
            if b.kind == "building":
                self.H1.append(torch.empty((N, b.ho, b.wo, f), dtype=BF16, device=dev))
                self.H2.append(None)
                self.Y1.append(None)
                self.Y2.append(None)
            else:
                self.H1.append(torch.empty((N, b.h, b.w, f), dtype=BF16, device=dev))
                self.H2.append(torch.empty((N, b.ho, b.wo, f), dtype=BF16, device=dev))
                for h, ys in ((self.H1[-1], self.Y1), (self.H2[-1], self.Y2)):
                    ys.append(torch.empty_like(h) if self._materialize_bn(h.numel() // f, f)
                              else None)
            self.X.append(torch.empty((N, b.ho, b.wo, b.cout), dtype=BF16, device=dev))
            if b.proj is not None:
                sc_max = max(sc_max, N * b.ho * b.wo * b.cout)
            max_act = max(max_act, N * b.h * b.w * b.cin, N * b.ho * b.wo * b.cout,
                          N * b.h * b.w * f)
        max_act = max(max_act, self.stem_out.numel())
        self.sc_buf = torch.empty(max(sc_max, 1), dtype=BF16, device=dev)
        self._gbufs = []
        F = spec.dense_in
        self.pooled = torch.empty((N, F), dtype=BF16, device=dev)
        self.dpooled = torch.empty((N, F), dtype=BF16, device=dev)
        self.logits = torch.empty((N, self.kpad), device=dev)
        self.dlogits = torch.empty((N, self.kpad), dtype=BF16, device=dev)
        # scratch: per-BN forward / backward partials (the BN's first consumer may combine
        # them -- BnPreFin / BnBwdPre -- while the same kernel produces the next BN's
        # partials, so no sharing), wgrad split-K slabs
        for b in self.bns.values():
            C = b.spec.channels
            M = N * b.spec.h * b.spec.w
            bm = min(self.nat.conv_gemm_bm(M, C), self.nat.bn_stats_tile_rows())
            b.part = torch.empty(_ceil(M, bm) * 2 * C, device=dev)
            tb = max(self.nat.bn_bwd_tiles(M, C), _ceil(M, self.nat.conv_gemm_bm(M, C)))
            b.bpart = torch.empty(tb * 2 * C, device=dev)
        # Accumulator mode (tune bn_acc, default on): the producing conv's workgroups add
        # their tile sums into BN_ACC_REP fp64 replicas per BatchNorm with memory-side
        # atomics, and the consumer reads 2 x REP values per channel instead of
        # combining every tile partial in its prologue or a finalize launch (measured on
        # the CIFAR direct convs: ~4 us per consumer prologue at 512 tiles).  All the
        # replicas live in one buffer zeroed by one memset at the start of the step.
        self.bn_acc_on = self.bn_bacc_on = bool(tune.get("bn_acc"))
        # (each BN's block holds the larger of the per-layer and the persistent kernels'
        # replica counts; a kernel uses the first replicas of the block)
        rep = max(self.nat.bn_acc_rep(), self.nat.prn_acc_rep())
        tot = sum(4 * rep * b.spec.channels for b in self.bns.values())
        # (+ N x 64 doubles and the barrier region: the persistent step's average-pool sums
        # and its sharded barrier counters / readiness line / item queue (128-B aligned lines),
        # zeroed with the accumulators at the start of every step -- train/persist.py)
        base = max(_ceil(tot, 2) * 2, 2)
        bar_d = _ceil(self.nat.prn_bar_words(), 2) + 16   # + up to 128 B of alignment
        self.bn_acc = torch.zeros(base + 64 * N + bar_d, dtype=torch.float64, device=dev)
        self.prn_pool = self.bn_acc.data_ptr() + 8 * base
        self.prn_bar = _ceil(self.bn_acc.data_ptr() + 8 * (base + 64 * N), 128) * 128
        off = 0
        for b in self.bns.values():
            n = 2 * rep * b.spec.channels
            b.acc = self.bn_acc[off:off + n]
            b.bacc = self.bn_acc[off + n:off + 2 * n]
            off += 2 * n
        max_c = max(b.spec.channels for b in self.bns.values())
        self.coef = torch.empty(3 * max_c, device=dev)
        # per-conv split-K partial slabs (persist until the bucket's grouped reduce)
        self.wg_off = {}
        tot = 0
        for name, c in self.convs.items():
            sp, pps = self.nat.wgrad_pick_splits(self._geom(c, N))
            self.wg_off[name] = (tot, sp, pps)
            g = self._geom(c, N)
            tot += sp * c.spec.cout * g[7] * g[8] * g[3]
        sp, pps = self.nat.wgrad_pick_splits(self._dense_geom(N))
        self.wg_off["dense"] = (tot, sp, pps)
        tot += sp * self.kpad * F
        self.wg_part = torch.empty(max(tot, 1), device=dev)
        self.l2_ws = torch.empty(self.nat.l2_workspace_floats(), device=dev)
        self.xent_ws = torch.empty(self.nat.softmax_xent_ws_floats(N, self.kpad), device=dev)

    # ------------------------------------------------------------------ helpers
    def _x_in_shape(self, N):
        H, W = self.spec.image_h, self.spec.image_w
        return (N, H // 2, W // 2, 16) if self.stem_s2d else (N, H, W, self.cpad_in)

    def _stem_input(self, x):
        """[N, H, W, C <= cpad] image batch -> the stem's operand layout (x_in)."""
        x = x.to(self.device)
        N, H, W, C = x.shape
        if self.stem_s2d:   # channel (rh * 2 + rw) * 4 + c of pixel (2q + rh, 2p + rw)
            if C > 4:       # an NHWC-8 (zero-padded) batch: its 3 image channels
                x, C = x[..., :3], 3
            xp = torch.zeros((N, H, W, 4), dtype=BF16, device=self.device)
            xp[..., :C] = x.to(BF16)
            return xp.view(N, H // 2, 2, W // 2, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(
                N, H // 2, W // 2, 16)
        if C != self.cpad_in:
            xp = torch.zeros((N, H, W, self.cpad_in), dtype=BF16, device=self.device)
            xp[..., :C] = x.to(BF16)
            return xp
        return x.to(BF16)

    def _geom(self, c: _Conv, N):
        s = c.spec
        if self.stem_s2d and s.name == self.spec.stem.name:
            return [N, s.h // 2, s.w // 2, 16, s.ho, s.wo, s.cout, 4, 4, 1, 2]
        return [N, s.h, s.w, c.cin, s.ho, s.wo, s.cout, s.kh, s.kw, s.stride, (s.kh - 1) // 2]

    def _dense_geom(self, N):
        return [N, 1, 1, self.spec.dense_in, 1, 1, self.kpad, 1, 1, 1, 0]

    def _consumer_cap(self, C: int) -> int:
        """Max partials a consumer prologue combines (bn_prefin_table / _sums)."""
        return self.nat.pfin_cap(C)

    def _conv_fwd(self, plan, c: _Conv, x, out, N, pre: _BN | None = None, residual=None,
                  stats_for: _BN | None = None):
        """One conv launch.  BatchNorm statistics of the output (``stats_for``) go
        into the BN's fp64 accumulators (bn_acc, default), which its first consumer
        reads; or, as per-tile partials, are finalized by the first consumer's prologue
        (few tiles) or else by a separate bn_finalize launch."""
        geom = self._geom(c, N)
        if self._fwd_stream(c, N, pre, stats_for):
            self._conv_fwd_stream(plan, c, x, out, N, pre, residual, stats_for)
            return
        stat_ptr = 0
        fin, pfin = [], []
        if pre is not None and pre.pending is not None:
            if pre.pending[0] == "acc":
                _, part, M0 = pre.pending
                cnt, rows = _ACC_CNT, 0
            else:
                part, cnt, rows, M0 = pre.pending
            pfin = [part, cnt, rows, M0, pre.gamma, pre.beta, pre.mean.data_ptr(),
                    pre.rstd.data_ptr(), pre.scale.data_ptr(), pre.shift.data_ptr(),
                    pre.mmean, pre.mvar]
            pre.pending = None
        if stats_for is not None:
            b = stats_for
            M, nc = N * c.spec.ho * c.spec.wo, c.spec.cout
            bm, bn = self.nat.conv_gemm_bm(M, nc), self.nat.conv_gemm_bn(M, nc)
            T = _ceil(M, bm)
            stat_ptr = b.part.data_ptr()
            b.pending = (stat_ptr, T, bm, M)
            # measured (CIFAR bs 128 / 32): the consumer prologue when the tiles are few,
            # else a separate finalize, beats producer-side last-arriver finalizes
            if self.bn_acc_on:
                fin = [b.acc.data_ptr()]
                b.pending = ("acc", b.acc.data_ptr(), M)
            elif T > self._consumer_cap(nc):
                b.pending = ("separate", stat_ptr, T, bm, M)
        plan.conv_gemm(0, x.data_ptr(), c.ohwi, out.data_ptr(), 0,
                       0 if residual is None else residual.data_ptr(),
                       0 if pre is None else pre.scale.data_ptr(),
                       0 if pre is None else pre.shift.data_ptr(), 0, 0, stat_ptr, 0, geom, [],
                       fin, [], pfin, [], BN_DECAY, BN_EPS, 1)

    def _fwd_stream(self, c: _Conv, N, pre: _BN | None, stats_for: _BN | None) -> bool:
        """Whether a forward conv takes the streaming narrow-K 1x1 kernel (bn_fwd1x1.hip):
        1x1 stride 1, K = 64..256 input channels, >= 256-wide output, statistics (if any) in
        fp64 accumulators, its BN prologue (if any) finalized or pending in accumulators."""
        s = c.spec
        if not tune.get("fwd1x1_stream") or self.stem_s2d and s.name == self.spec.stem.name:
            return False
        if s.kh != 1 or s.kw != 1 or s.stride != 1:
            return False
        if not self.nat.bnf1x1_covers(N * s.ho * s.wo, s.cout, c.cin):
            return False
        if stats_for is not None and not self.bn_acc_on:
            return False
        return pre is None or pre.pending is None or pre.pending[0] == "acc"

    def _conv_fwd_stream(self, plan, c: _Conv, x, out, N, pre, residual, stats_for):
        s = c.spec
        M = N * s.ho * s.wo
        pfin, ps, psh = [], 0, 0
        if pre is not None and pre.pending is not None:
            _, part, M0 = pre.pending
            pfin = [part, _ACC_CNT, 0, M0, pre.gamma, pre.beta, pre.mean.data_ptr(),
                    pre.rstd.data_ptr(), pre.scale.data_ptr(), pre.shift.data_ptr(),
                    pre.mmean, pre.mvar]
            pre.pending = None
        elif pre is not None:
            ps, psh = pre.scale.data_ptr(), pre.shift.data_ptr()
        acc = 0
        if stats_for is not None:
            acc = stats_for.acc.data_ptr()
            stats_for.pending = ("acc", acc, M)
        plan.bnf1x1([x.data_ptr(), c.ohwi, 0 if residual is None else residual.data_ptr(),
                     out.data_ptr(), ps, psh, acc], pfin, M, s.cout, c.cin, BN_DECAY, BN_EPS, 1)

    def _bn_input(self, plan, bn: _BN, x, y):
        """Operand of the conv consuming BN(x): (y, None) after materializing
        y = ReLU(BN(x)) when the plan gave the BN a buffer `y` (_alloc_activations),
        else (x, bn) -- the conv applies BN+ReLU while staging (PRE)."""
        if y is None:
            self._bn_finalize(plan, bn)
            return x, bn
        C = bn.spec.channels
        if bn.pending is not None and bn.pending[0] == "acc":
            # the apply pass finalizes too (no bn_finalize launch in between)
            _, part, M = bn.pending
            bn.pending = None
            plan.bn_relu_apply_acc(x.data_ptr(), y.data_ptr(), M, C, part, bn.gamma, bn.beta,
                                   bn.mmean, bn.mvar, BN_DECAY, BN_EPS, 1, bn.mean.data_ptr(),
                                   bn.rstd.data_ptr(), bn.scale.data_ptr(), bn.shift.data_ptr())
            return y, None
        self._bn_finalize(plan, bn, consumer_conv=False)
        plan.bn_relu_apply(x.data_ptr(), bn.scale.data_ptr(), bn.shift.data_ptr(), y.data_ptr(),
                           x.numel() // C, C)
        return y, None

    def _materialize_bn(self, M: int, C: int) -> bool:
        """Inner bottleneck BN: materialize ReLU(BN(x)) once instead of applying it in
        the consumer conv's A staging (PRE), whose VALU work is repeated by every
        output-column tile and, beside the MFMAs of the small 64x64 tiles of the 7x7
        layers, cost more than the MFMAs (3x3 512->512: 66 -> 103 us).  Materializing
        is one streaming pass: a win where the tensor is small and the consumers'
        column tiles many (tune mat_bn_elems: M*C threshold, 0 = never; mat_bn_minc: min
        channels).  Measured (RN50 bs128): stages 3-4 (14x14 / 7x7) +1.3 %; adding stage 2
        no gain."""
        return C >= tune.get("mat_bn_minc") and M * C <= tune.get("mat_bn_elems")

    def _bn_finalize(self, plan, bn: _BN, train=True, consumer_conv: bool = True):
        """Called where the BN's statistics are next needed.  Deferred to the first
        consumer conv when that conv can combine the partials itself (BnPreFin);
        otherwise (or for a non-conv consumer) one bn_finalize launch (case (d))."""
        if bn.pending is None:
            return
        if bn.pending[0] == "acc":
            if consumer_conv:
                return
            _, part, M = bn.pending
            tiles, rows = -1, 0
        elif bn.pending[0] == "separate":
            _, part, tiles, rows, M = bn.pending
        elif consumer_conv:
            return
        else:
            part, tiles, rows, M = bn.pending
        bn.pending = None
        plan.bn_finalize(part, tiles, rows, M, bn.spec.channels, bn.gamma,
                         bn.beta, bn.mmean, bn.mvar, BN_DECAY, BN_EPS, int(train),
                         bn.mean.data_ptr(), bn.rstd.data_ptr(), bn.scale.data_ptr(),
                         bn.shift.data_ptr())

    def _mark(self, plan, *names):
        idx = plan.size()
        for n in names:
            self.ready_index[n] = idx

    def _bap_ok(self, c: _Conv, N) -> bool:
        """Whether the first 1x1 dgrad of an identity bottleneck block emits its input
        BatchNorm's backward output itself (_conv_bwd ``bap``): accumulator-mode sums,
        a shape the streaming kernel covers, and the block's wide input channels within
        the ``bap_maxc`` bound (0 = off)."""
        s = c.spec
        maxc = tune.get("bap_maxc")
        if not (self.bn_bacc_on and maxc > 0 and c.cin <= maxc):
            return False
        if s.kh != 1 or s.kw != 1 or s.stride != 1:
            return False
        return (self.nat.bnd1x1_covers(N * s.h * s.w, c.cin, s.cout)
                and not self.nat.conv_direct_covers(1, self._geom(c, N)))

    def _dgrad_stream_ok(self, c: _Conv, N) -> bool:
        """1x1 stride-1 dgrads with BN-backward sums whose weights fit the streaming kernel
        (bn_dgrad1x1.hip mode 2): the expanding conv's dgrad at stages 1-2, the first
        conv's at stage 3 (tune dgrad1x1_stream)."""
        s = c.spec
        if not tune.get("dgrad1x1_stream") or s.kh != 1 or s.kw != 1 or s.stride != 1:
            return False
        M = N * s.h * s.w
        return (self.nat.bnd1x1_covers(M, c.cin, s.cout)
                and not self.nat.conv_direct_covers(1, self._geom(c, N)))

    def _conv_bwd(self, plan, c: _Conv, dy, x, N, pre: _BN | None, dx=None, accumulate=False,
                  bnb: tuple | None = None, side: bool = True, bap: tuple | None = None):
        """dgrad into dx (optional), then wgrad (+ reduce into the flat gradient).

        ``bnb=(bn, bn_input)``: the dgrad epilogue also emits that BN's backward
        partial sums (sum g, sum g*xhat of dx).  If ``dy`` is the output of a
        pending BN backward (_bn_bwd), the direct dgrad applies that BN backward
        while staging dy (BnBwdPre) and materializes dy for the wgrad.

        ``bap=(bn, add)`` (bn's input is ``x``, the 1x1 conv's own input): dx receives
        the BN+ReLU backward OUTPUT, BNbwd(dgrad) + add, with no separate apply pass.
        The dgrad runs twice on the streaming kernel (bn_dgrad1x1.hip): a first pass only
        sums (sum g, sum g*xhat into the fp64 accumulators, no store), a finalize turns
        the sums into the apply coefficients, and the second pass recomputes the same
        GEMM tile (bitwise the same fp32 values) and applies BN backward + add.
        For a bottleneck block's first conv the GEMM is narrow (K = 64..512 input
        rows), while the BN'd tensor is wide (256..2048 channels): recomputing it
        costs less than writing the wide gradient, re-reading it and x, and writing
        dx in a separate apply (reference: FusedBatchNormGrad after
        Conv2DBackpropInput, resnet_model_official.py:133-175)."""
        geom = self._geom(c, N)
        s = c.spec
        abw = []
        a_src = dy
        pb = self._pending_bwd
        if pb is not None:
            fuse = pb["out"] is dy and dx is not None
            # the direct (CIFAR) dgrad applies the pending BN backward while staging dy;
            # the implicit-GEMM dgrads keep the separate apply (fusing it there repeated
            # the per-element work per column tile and tap: ImageNet 13.3 -> 17.8 ms)
            if fuse and self.nat.conv_direct_covers(1, geom):
                bn = pb["bn"]
                add = pb["add"]
                part, cnt = pb["part"], pb["cnt"]
                if cnt != -1 and cnt > self._consumer_cap(s.cout):
                    # too many partials for the prologue: finalize separately, the
                    # dgrad then reads the coefficients (cnt = 0)
                    plan.bn_bwd_finalize(part, cnt, pb["M"], bn.spec.channels, bn.gamma,
                                         bn.rstd.data_ptr(), bn.dgamma, bn.dbeta,
                                         self.coef.data_ptr())
                    part, cnt = 0, 0
                abw = [pb["x"].data_ptr(), 0 if add is None else add.data_ptr(),
                       bn.mean.data_ptr(), bn.rstd.data_ptr(), bn.scale.data_ptr(),
                       bn.shift.data_ptr(), bn.gamma, part, _ACC_CNT if cnt == -1 else cnt,
                       dy.data_ptr(),
                       bn.dgamma, bn.dbeta, self.coef.data_ptr()]
                self._produced.update(bn.names)
                self._pending_bwd = None
                a_src = pb["da"]        # the dgrad stages BNbwd(da) and writes dy itself
            else:
                self._emit_bn_bwd(plan)
        if dx is not None and bap is not None:
            bn, add = bap
            self.n_bap += 1
            assert not abw, "bap: the dgrad's input is not a pending BN-backward output"
            M, C = N * s.h * s.w, c.cin
            bl = [x.data_ptr(), bn.mean.data_ptr(), bn.rstd.data_ptr(), bn.scale.data_ptr(),
                  bn.shift.data_ptr()]
            # the streaming kernel (bn_dgrad1x1.hip) runs both passes (_bap_ok checked coverage)
            base = [a_src.data_ptr(), c.hwio, x.data_ptr()]
            bnp = bl[1:]
            plan.bnd1x1(0, base + [0, 0] + bnp + [0, bn.bacc.data_ptr()], M, C, s.cout)
            plan.bn_bwd_finalize(bn.bacc.data_ptr(), -1, M, C, bn.gamma, bn.rstd.data_ptr(),
                                 bn.dgamma, bn.dbeta, self.coef.data_ptr())
            self._produced.update(bn.names)
            addp = 0 if add is None else add.data_ptr()
            plan.bnd1x1(1, base + [addp, dx.data_ptr()] + bnp + [self.coef.data_ptr(), 0], M, C,
                        s.cout)
        elif dx is not None:
            bl, bfl = [], []
            if bnb is not None:
                bn, bx = bnb
                Mx = N * s.h * s.w
                C = c.cin
                T = _ceil(Mx, self.nat.conv_gemm_bm(Mx, C))
                bl = [bx.data_ptr(), bn.mean.data_ptr(), bn.rstd.data_ptr(), bn.scale.data_ptr(),
                      bn.shift.data_ptr(), bn.bpart.data_ptr()]
                self._bnb_src = (bn.bpart.data_ptr(), T)
                if self.bn_bacc_on:
                    bfl = [bn.bacc.data_ptr()]
                    self._bnb_src = (bn.bacc.data_ptr(), -1)
            stream_bnb = (bnb is not None and self.bn_bacc_on and not accumulate and not abw
                          and self._dgrad_stream_ok(c, N))
            if stream_bnb and "dgrad" not in _DIAG_SKIP:
                # 1x1 dgrad + BN-backward sums on the streaming kernel (bn_dgrad1x1.hip mode 2)
                plan.bnd1x1(2, [a_src.data_ptr(), c.hwio, bx.data_ptr(), 0, dx.data_ptr()] +
                            bl[1:5] + [0, bn.bacc.data_ptr()], Mx, C, s.cout)
            elif "dgrad" not in _DIAG_SKIP:
                plan.conv_gemm(1, a_src.data_ptr(), c.hwio, dx.data_ptr(), 0, 0, 0, 0, 0, 0,
                               0, int(accumulate), geom, bl, [], bfl, [], abw, BN_DECAY, BN_EPS,
                               1)
        # The weight gradient only feeds the bucket's grouped reduce, so it runs on
        # the side stream, overlapping the dgrad -> BN-backward chain.  Forks are
        # batched per residual block (_flush_side): a cross-stream event pair costs
        # ~6 us of device time on ROCm, about a third of a CIFAR wgrad.
        off, sp, pps = self.wg_off[s.name]
        part = self.wg_part.data_ptr() + 4 * off

        desc = (dy.data_ptr(), x.data_ptr(), 0 if pre is None else pre.scale.data_ptr(),
                0 if pre is None else pre.shift.data_ptr(), part, tuple(geom), sp, pps)
        if self.fork_wgrad and side:
            self._side_q.append(desc)
        else:
            self._emit_wgrads(plan, [desc])
            # a side-stream reduce of this slab must fork after it (_flush_side)
            self._main_wgrad = self.fork_wgrad
        if self.stem_s2d and s.name == self.spec.stem.name:   # 4x4x16 HWIO, mapped back by _emit_reduce
            self._pending[c.name] = (part, self.stem_g4.data_ptr(), sp, s.cout, s.cout, 16, 16, 16)
        else:
            self._pending[c.name] = (part, c.grad, sp, s.cout, s.cout, s.kh * s.kw, c.cin,
                                     c.cin_valid)
        self._produced.add(c.name)

    def _bn_bwd(self, plan, bn: _BN, dy, x, dx, add=None, reduced: bool = False):
        """BN+ReLU backward dx = BNbwd(dy) (+ add).  ``reduced``: the producing dgrad
        already wrote the partial sums (conv epilogue BNB).  The finalize + apply are
        deferred: the next dgrad consuming dx applies them while staging its input
        (_conv_bwd), else _emit_bn_bwd launches them."""
        C = bn.spec.channels
        M = x.numel() // C
        if self._pending_bwd is not None:
            self._emit_bn_bwd(plan)
        if reduced:
            part, cnt = self._bnb_src
        else:
            cnt = self.nat.bn_bwd_tiles(M, C)
            part = bn.bpart.data_ptr()
            plan.bn_bwd_reduce(dy.data_ptr(), x.data_ptr(), bn.mean.data_ptr(),
                               bn.rstd.data_ptr(), bn.scale.data_ptr(), bn.shift.data_ptr(), M, C,
                               part)
        self._pending_bwd = dict(bn=bn, da=dy, x=x, out=dx, add=add, part=part, cnt=cnt, M=M)

    def _emit_bn_bwd(self, plan):
        """Launch the pending BN backward's finalize + apply (no fusing consumer)."""
        pb = self._pending_bwd
        if pb is None:
            return
        self._pending_bwd = None
        bn, M, C = pb["bn"], pb["M"], pb["bn"].spec.channels
        add = pb["add"]
        self._produced.update(bn.names)
        if pb["cnt"] == -1 and self.nat.bn_bwd_apply_acc_fits(M, C):
            # accumulator sums, small C: the apply launch finalizes too (one launch less)
            plan.bn_bwd_apply_acc(pb["da"].data_ptr(), pb["x"].data_ptr(), bn.mean.data_ptr(),
                                  bn.rstd.data_ptr(), bn.scale.data_ptr(), bn.shift.data_ptr(),
                                  [pb["part"], bn.gamma, bn.dgamma, bn.dbeta,
                                   self.coef.data_ptr()],
                                  0 if add is None else add.data_ptr(), pb["out"].data_ptr(), M, C)
            return
        plan.bn_bwd_finalize(pb["part"], pb["cnt"], M, C, bn.gamma, bn.rstd.data_ptr(),
                             bn.dgamma, bn.dbeta, self.coef.data_ptr())
        plan.bn_bwd_apply(pb["da"].data_ptr(), pb["x"].data_ptr(), bn.mean.data_ptr(),
                          bn.rstd.data_ptr(), bn.scale.data_ptr(), bn.shift.data_ptr(),
                          self.coef.data_ptr(), 0 if add is None else add.data_ptr(),
                          pb["out"].data_ptr(), M, C)

    def _flush_side(self, plan, force: bool = False):
        """Fork: emit the queued weight gradients on the side stream behind ONE event
        (every `fork_every` residual blocks, or now if `force`)."""
        if not self._side_q and not (force and self._main_wgrad):
            return
        self._side_blocks += 1
        if not force and self._side_blocks < self.fork_every:
            return
        self._main_wgrad = False   # the fork orders them before everything queued now
        ev = plan.new_event()
        plan.record(ev)
        plan.use_stream(1)
        plan.wait(ev)
        self._emit_wgrads(plan, self._side_q)
        plan.use_stream(0)
        self._side_q, self._side_blocks = [], 0

    def _split_tail_on(self) -> bool:
        return self.fork_wgrad and self.tail_main > 0

    def _split_tail(self, plan) -> list:
        """End of the dgrad chain (first block done): fork the first part of the queued
        weight gradients to the side stream now and return the last `tail_main`
        fraction, which the main stream runs after the stem instead of idling until the
        side stream drains them.  The bucket reduces are emitted afterwards (forced
        flush), so no reduce can read a slab before its main-stream wgrad."""
        q = self._side_q
        k = len(q) - int(round(self.tail_main * len(q)))
        while k < len(q) and callable(q[k]):   # queued non-wgrad side ops stay on the side
            k += 1
        self._side_q = q[:k]
        if self._side_q:
            self._flush_side(plan, force=True)
        else:
            self._side_blocks = 0
        return q[k:]

    def _emit_wgrads(self, plan, descs):
        """Weight-gradient launches on the current stream, in queue order (queued
        non-wgrad side ops -- the head's batch folds, the dense wgrad -- are callables)."""
        for d in descs:
            if callable(d):
                d()
            elif "wgrad" not in _DIAG_SKIP:   # (diagnostics only: scripts/diag_step.py)
                plan.conv_wgrad(d[0], d[1], d[2], d[3], d[4], list(d[5]), d[6], d[7])

    def _flush_buckets(self, plan, force: bool = False):
        """Emit the grouped split-K reduce of every reduce group whose gradients are
        all produced (all remaining ones if `force`).  A bucket whose groups are all
        reduced is ready for its all-reduce (world > 1): with the native communicator
        the comm stream waits on the main stream (BN parameter gradients) AND on the
        side stream (the bucket's reduces), so the main stream's dgrad chain never
        waits for the side stream mid-backward; for host-issued c10d all-reduces the
        side stream is joined into the main stream (the host issues on main).  With
        one process the only join is the final one."""
        for bi, (lo, hi, names) in enumerate(self.buckets):
            if bi in self._flushed:
                continue
            for gi, gnames in enumerate(self.reduce_groups[bi]):
                if (bi, gi) in self._reduced:
                    continue
                if not force and not all(n in self._produced for n in gnames):
                    continue
                self._flush_side(plan, force=True)   # the group's wgrads precede its reduce
                self._emit_reduce(plan, gnames)
                self._reduced.add((bi, gi))
            if not all((bi, gi) in self._reduced for gi in range(len(self.reduce_groups[bi]))):
                continue
            if self.comm is not None:
                self._mark(plan, *names)
                self._flushed.add(bi)
                self._emit_allreduce(plan, lo, hi,
                                     side_dep=self.fork_wgrad and not self._reduce_main)
                continue
            if self.reduce_buckets or force:
                if self.fork_wgrad and not self._reduce_main:
                    # join: the main stream (and the bucket's all-reduce) waits for the side stream
                    ev = plan.new_event()
                    plan.use_stream(1)
                    plan.record(ev)
                    plan.use_stream(0)
                    plan.wait(ev)
                self._mark(plan, *names)
                self._flushed.add(bi)

    def _emit_allreduce(self, plan, lo: int, hi: int, side_dep: bool, on_main: bool = False,
                        packed: bool = False):
        """Fork the comm stream off the main stream (and, with ``side_dep``, off the
        side stream, where the bucket's split-K reduces ran) at the bucket's ready
        point and all-reduce grad[lo:hi) there (bf16 exchange: cast kernels on the
        comm stream around a bf16 all-reduce), while the compute streams continue.
        ``on_main``: on the main stream itself, no fork and no join (the persistent
        step: nothing is left to overlap, and each event costs ~5 us between launches).
        ``packed``: grad_bf16[lo:hi) already holds the bf16 input (_emit_pack) and the
        optimizer reads the result from it: no cast launches."""
        if on_main:
            assert not side_dep
        else:
            evs = [plan.new_event()]
            plan.record(evs[0])
            if side_dep:
                evs.append(plan.new_event())
                plan.use_stream(1)
                plan.record(evs[1])
            plan.use_stream(2)
            for ev in evs:
                plan.wait(ev)
        n = hi - lo
        g = self.grad.data_ptr() + 4 * lo
        if self.grad_bf16 is not None:
            gb = self.grad_bf16.data_ptr() + 2 * lo
            if not packed:
                plan.cast_f32_bf16(g, gb, n)
            plan.all_reduce(self.comm, gb, n, self.nat.COMM_BF16)
            if not packed:
                plan.cast_bf16_f32(gb, g, n)
        else:
            plan.all_reduce(self.comm, g, n, self.nat.COMM_F32)
        self._n_allreduce += 1
        self._comm_forks += 0 if on_main else 1
        self._allreduce_bytes += n * (2 if self.grad_bf16 is not None else 4)
        plan.use_stream(0)

    def _join_comm(self, plan):
        """The optimizer (main stream) waits for every bucket's all-reduce."""
        if self.comm is None or not self._comm_forks:
            return
        ev = plan.new_event()
        plan.use_stream(2)
        plan.record(ev)
        plan.use_stream(0)
        plan.wait(ev)

    def _packed_gin(self) -> int:
        """The optimizer's gradient source after a packed all-reduce: grad_bf16 (bf16
        exchange) or grad itself (0: fp32 exchange, the pack summed the slabs into it)."""
        return self.grad_bf16.data_ptr() if self.grad_bf16 is not None else 0

    def _emit_pack(self, plan, names, stream: int = 0):
        """The all-reduce input of `names`' gradients in ONE launch (sgd_tiles pack mode,
        the optimizer's own slab summation): split-K slab sums and the other gradients as
        bf16 into grad_bf16 (fp32 exchange: the slab sums into grad).  Replaces a grouped
        reduce plus a cast launch; the optimizer then reads the all-reduced bf16 (gin)."""
        names = [n for n in names]
        slabs = {n: self._pending.pop(n) for n in names if n in self._pending}
        wt, bt, nblk = self._sgd_tiles_work(slabs, names=set(names))
        s = self.sched
        gout = self.grad_bf16.data_ptr() if self.grad_bf16 is not None else 0
        plan.use_stream(stream)
        plan.sgd_tiles(self.params.master.data_ptr(), self.grad.data_ptr(), self.mom.data_ptr(),
                       s.init, s.warm_steps, s.warm_from, s.warm_to, list(s.bounds),
                       list(s.values), self.gstep.data_ptr(), self.momentum, self.wd, 1.0,
                       int(self.use_momentum), self.segs.data_ptr(), wt.data_ptr(), bt.data_ptr(),
                       nblk, self.wbf.data_ptr(), 0, 0, 0, gout, 1)
        plan.use_stream(0)

    def _emit_reduce(self, plan, names, stream: int | None = None):
        descs = [self._pending.pop(n) for n in names if n in self._pending]
        if not descs:
            return
        arr = np.zeros(len(descs), dtype=WGD_DTYPE)
        chunk = 0
        for i, (part, grad, sp, K, Kv, taps, C, Cv) in enumerate(descs):
            arr[i] = (part, grad, sp, K, Kv, taps, C, Cv, chunk)
            chunk += self.nat.wgrad_reduce_chunks(sp, K, taps, C)
        t = torch.from_numpy(arr.view(np.uint8).copy()).to(self.device)
        self._keep.append(t)
        if stream is None:
            stream = 1 if self.fork_wgrad and not self._reduce_main else 0
        plan.use_stream(stream)
        plan.wgrad_reduce_grouped(t.data_ptr(), len(descs), chunk, 1.0)
        st = self.spec.stem
        sc = self.convs[st.name]
        if self.stem_s2d and sc.name in names:   # names: slot names ("conv2d/kernel")
            plan.stem_s2d_grad(self.stem_g4.data_ptr(), sc.grad, st.cout)
        plan.use_stream(0)

    def _g(self, i, shape):
        """A fresh gradient buffer per backward tensor (the index is ignored):
        with weight gradients running on the side stream, a rotating pool would
        need WAR fences; 288 GB of HBM makes per-tensor buffers the simpler choice."""
        t = torch.empty(shape, dtype=BF16, device=self.device)
        self._gbufs.append(t)
        return t

    # ------------------------------------------------------------------ plan
    def _build_train_plan(self):
        if self.persist:
            return self._build_persist_plan()
        plan, spec, N = self.plan, self.spec, self.N
        self.seg = {}
        for e in self.bns.values():
            e.pending = None
        self._n_allreduce, self._allreduce_bytes, self._comm_forks = 0, 0, 0
        b0 = plan.size()
        self._t_fwd0 = plan.timing_point("fwd_begin")
        # the step's BN accumulators start at zero: cleared by the CIFAR augmentation
        # kernel (no extra launch), else by a memset
        zero = (self.bn_acc.data_ptr(), self.bn_acc.numel() * 8) \
            if (self.bn_acc_on or self.bn_bacc_on) else (0, 0)
        if zero[0] and self.input_mode not in ("cifar_u8", "imagenet_u8"):
            plan.memset(*zero)
        # ---- input
        if self.input_mode == "cifar_u8":
            plan.cifar_augment(self.img_u8.data_ptr(), self.x_in.data_ptr(), N, spec.image_h,
                               spec.image_w, self.cpad_in, 4, self.data_seed,
                               self.gstep.data_ptr(), 1, 0, *zero)
        elif self.input_mode == "imagenet_u8":
            plan.imagenet_u8_pack(self.img_u8.data_ptr(), self.x_in.data_ptr(), N, spec.image_h,
                                  spec.image_w, self.data_seed, self.gstep.data_ptr(), 1, *zero,
                                  int(self.stem_s2d))
        # ---- forward
        stem = self.convs[spec.stem.name]
        blocks = spec.blocks
        first_bn = self.bns[blocks[0].bns[0].name]
        if spec.maxpool:
            self._conv_fwd(plan, stem, self.x_in, self.stem_out, N)
            st = spec.stem
            ph = _ceil(st.ho, 2)
            pad = max((ph - 1) * 2 + 3 - st.ho, 0) // 2
            plan.maxpool_fwd(self.stem_out.data_ptr(), self.pool_out.data_ptr(),
                             self.pool_arg.data_ptr(),
                             [N, st.ho, st.wo, st.cout, ph, ph, st.cout, 3, 3, 2, pad], 3)
            M = N * ph * ph
            plan.bn_stats(self.pool_out.data_ptr(), M, st.cout, first_bn.part.data_ptr())
            T = self.nat.bn_bwd_tiles(M, st.cout)
            rows = self.nat.bn_stats_tile_rows()
            first_bn.pending = (first_bn.part.data_ptr(), T, rows, M)
            if T > self._consumer_cap(st.cout):
                first_bn.pending = ("separate",) + first_bn.pending
        else:
            self._conv_fwd(plan, stem, self.x_in, self.stem_out, N, stats_for=first_bn)
        for i, b in enumerate(blocks):
            X, Xn = self.X[i], self.X[i + 1]
            bns = [self.bns[s.name] for s in b.bns]
            convs = [self.convs[c.name] for c in b.convs]
            nxt = self.bns[blocks[i + 1].bns[0].name] if i + 1 < len(blocks) else \
                self.bns[spec.final_bn.name]
            self._bn_finalize(plan, bns[0])
            residual = X
            if b.proj is not None:
                pc = self.convs[b.proj.name]
                sc = self.sc_buf[:N * b.ho * b.wo * b.cout].view(N, b.ho, b.wo, b.cout)
                self._conv_fwd(plan, pc, X, sc, N, pre=bns[0])
                residual = sc
            if b.kind == "building":
                self._conv_fwd(plan, convs[0], X, self.H1[i], N, pre=bns[0], stats_for=bns[1])
                self._bn_finalize(plan, bns[1])
                self._conv_fwd(plan, convs[1], self.H1[i], Xn, N, pre=bns[1], residual=residual,
                               stats_for=nxt)
            else:
                self._conv_fwd(plan, convs[0], X, self.H1[i], N, pre=bns[0], stats_for=bns[1])
                a1, p1 = self._bn_input(plan, bns[1], self.H1[i], self.Y1[i])
                self._conv_fwd(plan, convs[1], a1, self.H2[i], N, pre=p1, stats_for=bns[2])
                a2, p2 = self._bn_input(plan, bns[2], self.H2[i], self.Y2[i])
                self._conv_fwd(plan, convs[2], a2, Xn, N, pre=p2, residual=residual,
                               stats_for=nxt)
        fbn = self.bns[spec.final_bn.name]
        XL = self.X[-1]
        HL, WL, F = XL.shape[1], XL.shape[2], XL.shape[3]
        sp = self.scalars.data_ptr()
        # Small (CIFAR) heads: ONE launch for final BN finalize + BN-ReLU-avgpool + dense +
        # softmax-xent rows + dense dgrad + avgpool backward + the final BN's backward
        # sums (head_fused, head.hip) instead of 8 dependent launches; the batch folds
        # (loss, precision, dbias) and the dense wgrad go to the side stream.
        self._head_fused = (self.bn_acc_on and self.bn_bacc_on and fbn.pending is not None
                            and fbn.pending[0] == "acc" and bool(tune.get("fused_head"))
                            and self.nat.head_fused_supported(N, HL * WL, F, spec.num_classes,
                                                              self.kpad))
        self._dact = self._g(0, (N, HL, WL, F))
        if self._head_fused:
            fbn.pending = None
            plan.head_fused(XL.data_ptr(),
                            [fbn.acc.data_ptr(), fbn.gamma, fbn.beta, fbn.mmean, fbn.mvar,
                             fbn.mean.data_ptr(), fbn.rstd.data_ptr(), fbn.scale.data_ptr(),
                             fbn.shift.data_ptr()], BN_DECAY, BN_EPS, 1, self.dense_hwio,
                            self.dense_bias, self.labels.data_ptr(),
                            [N, HL * WL, F, spec.num_classes, self.kpad], 1.0 / self.global_batch,
                            [self.pooled.data_ptr(), self.dlogits.data_ptr(),
                             self.xent_ws.data_ptr(), self._dact.data_ptr(),
                             fbn.bacc.data_ptr()])
        else:
            self._bn_finalize(plan, fbn, consumer_conv=False)   # consumer: bnrelu_avgpool
            plan.bnrelu_avgpool(XL.data_ptr(), fbn.scale.data_ptr(), fbn.shift.data_ptr(),
                                self.pooled.data_ptr(), N, HL * WL, F)
            plan.conv_gemm(0, self.pooled.data_ptr(), self.dense_ohwi, 0, self.logits.data_ptr(),
                           0, 0, 0, self.dense_bias, spec.num_classes, 0, 0, self._dense_geom(N),
                           [], [], [], [], [], BN_DECAY, BN_EPS, 1)
            plan.softmax_xent(self.logits.data_ptr(), self.kpad, self.labels.data_ptr(), N,
                              spec.num_classes, sp, sp + 4, self.dlogits.data_ptr(),
                              self.dense_bias_grad, 1.0 / self.global_batch, 0,
                              self.xent_ws.data_ptr())
        self.seg["fwd"] = (b0, plan.size())

        # ---- backward
        b1 = plan.size()
        self._t_bwd0 = plan.timing_point("bwd_begin")
        self._pending, self._produced, self._flushed = {}, {"dense/bias"}, set()
        self._reduced = set()
        self._side_q, self._side_blocks = [], 0
        # the dense wgrad below runs on the main stream (unless the head is fused)
        self._main_wgrad = self.fork_wgrad and not self._head_fused
        self._pending_bwd, self._bnb_src = None, None
        self._reduce_main = False
        self.n_bap = 0   # identity blocks whose first dgrad applies its BN backward (bap)
        dg = self._dense_geom(N)
        off, spl, pps = self.wg_off["dense"]
        dpart = self.wg_part.data_ptr() + 4 * off
        dense_wgrad = lambda: plan.conv_wgrad(self.dlogits.data_ptr(),  # noqa: E731
                                              self.pooled.data_ptr(), 0, 0, dpart, dg, spl, pps)
        self._pending[self.dense_name] = (dpart, self.dense_grad, spl, self.kpad,
                                          spec.num_classes, 1, F, F)
        self._produced.add(self.dense_name)
        dact = self._dact
        d = 1
        dout = self._g(d, tuple(XL.shape))
        if self._head_fused:
            # batch folds of the head's rows (loss, precision, dbias) and the dense
            # weight gradient: side stream; the final BN backward is pending on its
            # accumulator sums for the first dgrad's BN-backward prologue
            xr = lambda: plan.softmax_xent_reduce(  # noqa: E731
                self.xent_ws.data_ptr(), self.kpad, N, spec.num_classes, sp, sp + 4,
                self.dense_bias_grad)
            if self.fork_wgrad:
                self._side_q += [xr, dense_wgrad]
            else:
                xr()
                dense_wgrad()
            self._bnb_src = (fbn.bacc.data_ptr(), -1)
            self._bn_bwd(plan, fbn, dact, XL, dout, reduced=True)
        else:
            dense_wgrad()
            plan.conv_gemm(1, self.dlogits.data_ptr(), self.dense_hwio, self.dpooled.data_ptr(), 0,
                           0, 0, 0, 0, 0, 0, 0, dg, [], [], [], [], [], BN_DECAY, BN_EPS, 1)
            plan.avgpool_bwd(self.dpooled.data_ptr(), dact.data_ptr(), N, HL * WL, F)
            self._bn_bwd(plan, fbn, dact, XL, dout)
        main_tail = []
        for i in range(len(blocks) - 1, -1, -1):
            b = blocks[i]
            X = self.X[i]
            bns = [self.bns[s.name] for s in b.bns]
            convs = [self.convs[c.name] for c in b.convs]
            o1, o2 = [j for j in range(3) if j != d]
            if b.kind == "building":
                h1 = self.H1[i]
                da = self._g(o1, tuple(h1.shape))
                self._conv_bwd(plan, convs[1], dout, h1, N, bns[1], dx=da, bnb=(bns[1], h1))
                dh = self._g(o2, tuple(h1.shape))
                self._bn_bwd(plan, bns[1], da, h1, dh, reduced=True)
                dcur = dh
            else:
                h1, h2 = self.H1[i], self.H2[i]
                # wgrad inputs: the materialized BN-ReLU output, or the BN input + PRE
                a1, p1 = (self.Y1[i], None) if self.Y1[i] is not None else (h1, bns[1])
                a2, p2 = (self.Y2[i], None) if self.Y2[i] is not None else (h2, bns[2])
                da = self._g(o1, tuple(h2.shape))
                self._conv_bwd(plan, convs[2], dout, a2, N, p2, dx=da, bnb=(bns[2], h2))
                dh2 = self._g(o2, tuple(h2.shape))
                self._bn_bwd(plan, bns[2], da, h2, dh2, reduced=True)
                da = self._g(o1, tuple(h1.shape))
                self._conv_bwd(plan, convs[1], dh2, a1, N, p1, dx=da, bnb=(bns[1], h1))
                dh1 = self._g(o2, tuple(h1.shape))
                self._bn_bwd(plan, bns[1], da, h1, dh1, reduced=True)
                dcur = dh1
            proj = b.proj is not None
            dx = self._g(o2, tuple(X.shape))
            if not proj and b.kind != "building" and self._bap_ok(convs[0], N):
                # identity bottleneck: conv1's dgrad emits BNbwd(.) + dout itself
                self._conv_bwd(plan, convs[0], dcur, X, N, bns[0], dx=dx, bap=(bns[0], dout))
            else:
                da1 = self._g(o1, tuple(X.shape))
                self._conv_bwd(plan, convs[0], dcur, X, N, bns[0], dx=da1,
                               bnb=None if proj else (bns[0], X))
                if proj:
                    self._conv_bwd(plan, self.convs[b.proj.name], dout, X, N, bns[0], dx=da1,
                                   accumulate=True, bnb=(bns[0], X))
                self._bn_bwd(plan, bns[0], da1, X, dx, add=None if proj else dout, reduced=True)
            dout, d = dx, o2
            if i == 0 and self._split_tail_on():
                main_tail = self._split_tail(plan)
                continue
            # the last block's weight gradients go out now so they overlap the stem's
            # backward (max-pool gather) instead of queueing behind it
            self._flush_side(plan, force=i == 0)
            self._flush_buckets(plan)
        # stem (no dgrad: the input needs no gradient)
        self._emit_bn_bwd(plan)     # the stem's consumers (maxpool_bwd / wgrad) are not fusing
        if spec.maxpool:
            dstem = self._g((d + 1) % 3, tuple(self.stem_out.shape))
            st = spec.stem
            ph = _ceil(st.ho, 2)
            pad = max((ph - 1) * 2 + 3 - st.ho, 0) // 2
            plan.maxpool_bwd(self.pool_arg.data_ptr(), dout.data_ptr(), dstem.data_ptr(),
                             [N, st.ho, st.wo, st.cout, ph, ph, st.cout, 3, 3, 2, pad], 3)
            dstem_src = dstem
        else:
            dstem_src = dout
        # The stem's weight gradient is the main stream's last op (nothing else is
        # left for it), running alongside the side stream's last weight gradients.
        self._conv_bwd(plan, stem, dstem_src, self.x_in, N, None, side=False)
        if main_tail:   # the main stream's share of the tail; the reduces fork after it
            self._emit_wgrads(plan, main_tail)
            self._main_wgrad = True
        if self._split_tail_on() and self.reduce_main_tail:
            # the remaining reduces run on the main stream after ONE join of the side
            # stream, instead of a fork to the side and a join back per bucket
            self._flush_side(plan, force=False)   # (the queue is empty after the split)
            ev = plan.new_event()
            plan.use_stream(1)
            plan.record(ev)
            plan.use_stream(0)
            plan.wait(ev)
            self._main_wgrad = False
            self._reduce_main = True
        self._flush_side(plan, force=True)
        self._flush_buckets(plan, force=True)
        self._t_bwd_done = plan.timing_point("bwd_compute_done")
        self._join_comm(plan)
        self._t_joined = plan.timing_point("allreduce_joined")
        self.seg["bwd"] = (b1, plan.size())

        self._emit_optimizer(plan)

    def _sgd_tiles_work(self, slabs, names=None, nosplit=(64, 64)):
        """The work map of the one-launch optimizer (csrc/optim.hip sgd_tiles_kernel): per
        parameter segment its slab (split-K partials still to be summed, or none: the
        gradient is in `grad`) and its first workgroup; weights with bf16 copies or slabs
        go in tiles of their HWIO master (opt_tile), other tensors in 1024-element chunks.
        `names`: only those segments get workgroups (a bucket's pack launch)."""
        work = np.zeros(self.nseg, dtype=OPTW_DTYPE)
        blk = []
        gptr = self.grad.data_ptr()
        for i, (rec, name) in enumerate(zip(self.seg_arr, self.seg_names)):
            if names is not None and name not in names:
                continue
            d = slabs.get(name)
            taps, C, K = int(rec["kh"] * rec["kw"]), int(rec["C"]), int(rec["K"])
            tiled = d is not None or rec["bf_ohwi"] >= 0 or rec["bf_hwio"] >= 0
            part, splits, kslab, cslab = 0, 0, 0, 0
            if d is not None:
                part, grad, splits, kslab, Kv, dtaps, cslab, Cv = d
                assert (grad, Kv, dtaps, Cv) == (gptr + 4 * int(rec["offset"]), K, taps, C), name
                assert kslab >= K and cslab >= C and part % 16 == 0, name
            tr = tc = 0
            if tiled:
                assert taps * C * K == rec["numel"], name
                tr, tc = opt_tile(taps * C, K, splits, cslab or C, C, taps, nosplit)
                n = _ceil(taps * C, tr) * _ceil(K, tc)
            else:
                n = _ceil(int(rec["numel"]), 1024)
            work[i] = (part, len(blk), splits, kslab, cslab, int(tiled), tr, tc)
            blk += [i] * n
        assert OPTW_DTYPE.itemsize == self.nat.opt_work_bytes()
        assert not set(slabs) - set(self.seg_names), "slab without a parameter segment"
        assert names is None or not set(slabs) - set(names), "slab outside the packed segments"
        wt = torch.from_numpy(work.view(np.uint8).copy()).to(self.device)
        bt = torch.tensor(blk, dtype=torch.int32, device=self.device)
        self._keep += [wt, bt]
        return wt, bt, len(blk)

    def _emit_update(self, plan, names, gin=0, step=True):
        """ONE sgd_tiles launch updating the segments `names` (no slabs: the gradient is in
        grad, or the all-reduced bf16 `gin`); step: it also does global_step += 1 (the
        step's last update launch)."""
        s = self.sched
        # (reading the all-reduced bf16, nothing to sum: 32 x 64 tiles, twice the
        # workgroups of 64 x 64 for a launch that is all load latency)
        wt, bt, nblk = self._sgd_tiles_work({}, names=names, nosplit=(32, 64) if gin else (64, 64))
        if not hasattr(self, "opt_ticket"):
            self.opt_ticket = torch.zeros(1, dtype=torch.int32, device=self.device)
        plan.sgd_tiles(self.params.master.data_ptr(), self.grad.data_ptr(), self.mom.data_ptr(),
                       s.init, s.warm_steps, s.warm_from, s.warm_to, list(s.bounds),
                       list(s.values), self.gstep.data_ptr(), self.momentum, self.wd, 1.0,
                       int(self.use_momentum), self.segs.data_ptr(), wt.data_ptr(), bt.data_ptr(),
                       nblk, self.wbf.data_ptr(), self.scalars.data_ptr() + 8,
                       self.opt_ticket.data_ptr() if step else 0, gin, 0, 0)

    def _emit_optimizer(self, plan, fused_slabs=None, gin=0, names=None):
        """Optimizer segment (fused SGD-momentum + wd + bf16 re-pack, global_step += 1)
        and the `cost` segment (1/2 sum v^2 of the weights).  fused_slabs (a dict, the
        persistent step): ONE sgd_tiles launch that also sums those weights' slabs.
        gin: the gradient is read from that bf16 buffer (the all-reduced pack, _emit_pack).
        names: only those segments (the rest were updated ahead, _emit_update)."""
        spec = self.spec
        sp = self.scalars.data_ptr()
        b2 = plan.size()
        s = self.sched
        if names is not None:
            assert not fused_slabs
            self._emit_update(plan, names, gin)
        elif fused_slabs is not None:
            # (reading the all-reduced bf16, nothing to sum: 32 x 64 tiles, twice the
            # workgroups of 64 x 64 for a launch that is all load latency)
            wt, bt, nblk = self._sgd_tiles_work(fused_slabs, nosplit=(32, 64) if gin else (64, 64))
            if not hasattr(self, "opt_ticket"):
                self.opt_ticket = torch.zeros(1, dtype=torch.int32, device=self.device)
            plan.sgd_tiles(self.params.master.data_ptr(), self.grad.data_ptr(),
                           self.mom.data_ptr(), s.init, s.warm_steps, s.warm_from, s.warm_to,
                           list(s.bounds), list(s.values), self.gstep.data_ptr(), self.momentum,
                           self.wd, 1.0, int(self.use_momentum), self.segs.data_ptr(),
                           wt.data_ptr(), bt.data_ptr(), nblk, self.wbf.data_ptr(), sp + 8,
                           self.opt_ticket.data_ptr(), gin, 0, 0)   # + global_step += 1
        else:
            plan.sgd_update_pack(self.params.master.data_ptr(), self.grad.data_ptr(),
                                 self.mom.data_ptr(), self.params.n_train, s.init, s.warm_steps,
                                 s.warm_from, s.warm_to, list(s.bounds), list(s.values),
                                 self.gstep.data_ptr(), self.momentum, self.wd, 1.0,
                                 int(self.use_momentum), self.segs.data_ptr(), self.nseg,
                                 self.wbf.data_ptr(), sp + 8, 1)
            plan.ohwi_pack(self.params.master.data_ptr(), self.segs.data_ptr(),
                           self.ohwi_tile0.data_ptr(), self.nseg, self.ohwi_tiles,
                           self.wbf.data_ptr(), self.gstep.data_ptr())   # + global_step += 1
        if self.stem_s2d:
            plan.stem_s2d_pack(self.stem_master, self.stem_w4.data_ptr(), spec.stem.cout)
        self._t_opt_end = plan.timing_point("opt_end")
        self.seg["opt"] = (b2, plan.size())
        # 1/2 sum v^2 of the weights, which only feeds the logged `cost`
        # (resnet_model.py:85-86; the gradient's wd*v is fused into the optimizer):
        # its own segment, run before the forward of the steps whose metrics are read
        # (step(need_cost=True); ImageNet RN50: 25.5 M floats, ~0.1 ms per step saved
        # on every other step).
        b3 = plan.size()
        plan.l2_half_sum(self.params.master.data_ptr(), self.params.n_train,
                         self.l2_ws.data_ptr(), sp + 12)
        self.seg["cost"] = (b3, plan.size())
        missing = [s.name for s in self.params.train_slots if s.name not in self.ready_index]
        assert not missing, f"gradients never produced: {missing[:4]}"

    def _build_persist_plan(self):
        """The persistent small-batch step (train/persist.py): input, ONE forward launch;
        ONE backward launch (dgrad chain + BN backward on the image row-slice workgroups,
        the weight gradients on the remaining CUs); the head's batch folds; on one GPU
        the optimizer launch (sum of the weight-gradient slabs included), else the
        grouped slab reduce, ONE all-reduce and the optimizer."""
        plan, spec, N = self.plan, self.spec, self.N
        self.seg = {}
        for e in self.bns.values():
            e.pending = None
        self._n_allreduce, self._allreduce_bytes, self._comm_forks = 0, 0, 0
        self._head_fused = False
        b0 = plan.size()
        self._t_fwd0 = plan.timing_point("fwd_begin")
        # BN accumulators, the pool sums and the two barrier counters start every step at zero
        zero = (self.bn_acc.data_ptr(), self.bn_acc.numel() * 8)
        if self.input_mode == "cifar_u8":
            plan.cifar_augment(self.img_u8.data_ptr(), self.x_in.data_ptr(), N, spec.image_h,
                               spec.image_w, self.cpad_in, 4, self.data_seed,
                               self.gstep.data_ptr(), 1, 0, *zero)
        else:
            plan.memset(*zero)
        ptrs, ints, floats = self.prn.args(self.prn_pool, self.prn_bar, BN_DECAY, BN_EPS, fwd=True)
        plan.prn(0, ptrs, ints, floats)
        ptrs, ints, floats = self.prn.args(self.prn_pool, self.prn_bar, BN_DECAY, BN_EPS)
        self.seg["fwd"] = (b0, plan.size())

        b1 = plan.size()
        self._t_bwd0 = plan.timing_point("bwd_begin")
        self._pending = dict(self.prn.pending())
        self._produced = set(self._pending) | {"dense/bias"}
        self._flushed, self._reduced = set(), set()
        self._side_q, self._side_blocks = [], 0
        self._main_wgrad = False
        self._reduce_main = True   # the slab reduces run on the main stream
        self._produced.add(self.dense_name)
        if self.prn.overlap:
            early = self._emit_persist_overlap(plan, ptrs, ints, floats)
            self.seg["bwd"] = (b1, plan.size())
            if self.opt_fused:   # the rest: the last bucket's segments
                self._emit_optimizer(plan, fused_slabs={}, gin=self._packed_gin(),
                                     names={n for n in self.seg_names if n not in early})
            else:
                self._emit_optimizer(plan)
            return
        plan.prn(1, ptrs, ints, floats)
        # the head's batch folds (loss, precision, dense bias and weight gradients): one
        # workgroup on the main stream -- no side stream, no fork/join events
        plan.prn(2, ptrs, ints, floats)
        # every slab is complete when the backward launch ends, and that launch holds
        # every CU (nothing can overlap it): ONE grouped reduce of all the slabs, then
        # (world > 1) ONE all-reduce of the whole gradient -- the per-bucket launches of
        # the per-layer plan only pay off when they overlap a backward (bs16: 6 reduce
        # launches 32 us vs 1).  With nothing to all-reduce and opt_fused, the slabs are
        # summed by the optimizer launch itself (sgd_tiles).
        all_names = [n for (_, _, names) in self.buckets for n in names]
        slabs = None
        packed = self.comm is not None and self.opt_fused
        if self.opt_fused and not self.reduce_buckets:
            slabs = {n: self._pending.pop(n) for n in all_names if n in self._pending}
        elif packed:   # the all-reduce input in one launch, read back by the optimizer
            self._emit_pack(plan, all_names)
        else:
            self._emit_reduce(plan, all_names)
        for bi, (lo, hi, names) in enumerate(self.buckets):
            self._mark(plan, *names)
            self._flushed.add(bi)
        if self.comm is not None:
            self._emit_allreduce(plan, min(b[0] for b in self.buckets),
                                 max(b[1] for b in self.buckets), side_dep=False, on_main=True,
                                 packed=packed)
        self._t_bwd_done = plan.timing_point("bwd_compute_done")
        self._join_comm(plan)
        self._t_joined = plan.timing_point("allreduce_joined")
        self.seg["bwd"] = (b1, plan.size())
        self._emit_optimizer(plan, fused_slabs=(slabs or {}) if self.opt_fused else None,
                             gin=self._packed_gin() if packed else 0)
        if slabs:
            # not part of the step: the slab sums alone, for callers that want this
            # step's gradient without the update (forward_backward)
            b4 = plan.size()
            self._pending.update(slabs)
            self._emit_reduce(plan, list(slabs))
            self.seg["gsum"] = (b4, plan.size())

    def _emit_persist_overlap(self, plan, ptrs, ints, floats):
        """World > 1: the persistent backward launch on the main stream, and on the comm
        stream (forked before it): the head's batch folds, then per gradient bucket but the
        last, in the order the backward completes them (persist.bucket_ranges), a one-wave
        wait for the bucket's line in the launch's barrier region to reach its count, the
        bucket's pack (or grouped slab reduce), its all-reduce and (opt_fused) the update of
        its parameters -- all while the backward still runs on the CUs left out of its
        grid.  The main stream joins the comm stream right after the backward (its buckets
        are long done by then) and packs, all-reduces and updates the last bucket itself.
        The stream check takes each bucket wait as a PARTIAL dependency on the backward
        launch (device_deps with the buffers it covers: the bucket's gradients / slabs and
        parameters, which the launch publishes complete and no longer reads once the count
        is reached, plus the lr slot and global step the launch never touches), and holds
        every comm-stream op before the join to the buffers it declares (op_buffers, R5).
        Returns the segment names updated on the comm stream."""
        from .persist import bucket_ranges

        fork = plan.new_event()
        plan.record(fork)
        plan.use_stream(2)
        plan.wait(fork)
        plan.prn(2, ptrs, ints, floats)        # head folds (loss, precision, dense grads)
        plan.use_stream(0)
        bwd_op = plan.size()
        plan.prn(1, ptrs, ints, floats)        # backward: dgrad chain + weight gradients
        err = self.prn.err.data_ptr()
        ranges = bucket_ranges(self)

        def declare(a0, bset):
            for i in range(a0, plan.size()):
                self._op_buffers[i] = set(bset)

        def bucket(b, lo, hi, names, stream):
            a0 = plan.size()
            if self.opt_fused:
                self._emit_pack(plan, names, stream=stream)
            else:
                self._emit_reduce(plan, names, stream=stream)
            plan.use_stream(stream)
            self._mark(plan, *names)
            self._emit_allreduce(plan, lo, hi, side_dep=False, on_main=True, packed=self.opt_fused)
            declare(a0, {f"grad:{b}"})

        early = set()
        for b, (lo, hi, names) in enumerate(ranges[:-1]):
            plan.use_stream(2)                 # (_emit_reduce/_emit_allreduce end on main)
            self._device_deps[plan.size()] = (bwd_op, {f"grad:{b}", f"param:{b}", "lr", "gstep"})
            plan.prn_bucket_wait(self.prn_bar, b, self.prn.bucket_target(b), err)
            bucket(b, lo, hi, names, 2)
            if self.opt_fused:
                # the bucket's parameters updated right behind its all-reduce, still beside
                # the backward: it has finished with them (their stage's dgrads and BN
                # backwards precede the count that released this bucket); global_step is
                # stepped by the last update launch
                plan.use_stream(2)
                a0 = plan.size()
                self._emit_update(plan, set(names), self._packed_gin(), step=False)
                declare(a0, {f"grad:{b}", f"param:{b}", "lr", "gstep"})
                plan.use_stream(0)
                early |= set(names)
        join = plan.new_event()
        plan.use_stream(2)
        plan.record(join)
        plan.use_stream(0)
        plan.wait(join)
        self._t_bwd_done = plan.timing_point("bwd_compute_done")
        bucket(len(ranges) - 1, *ranges[-1], 0)   # the last bucket behind the backward, in order
        for bi in range(len(self.buckets)):
            self._flushed.add(bi)
        self._t_joined = plan.timing_point("allreduce_joined")
        return early

    def forward_backward(self, st=None):
        """Forward + backward of the current batch with `grad` complete and no update
        (the persistent step on one GPU otherwise leaves its weight-gradient slabs to
        the optimizer launch)."""
        if self.persist_overlap:
            # the overlap plan updates the early buckets' parameters on the comm stream
            # inside the backward segment: no update-free backward exists
            raise RuntimeError("forward_backward: the persistent overlap plan (world > 1, "
                               "tune persist_overlap=1) updates parameters during the backward")
        st = torch.cuda.current_stream().cuda_stream if st is None else st
        self._run("fwd", st)
        self._run_bwd(st)
        if "gsum" in self.seg:
            self._run("gsum", st)

    def persist_error(self) -> bool:
        """Whether a persistent launch's barrier wait ever timed out (synchronises)."""
        return self.prn is not None and bool(self.prn.err.item())

    def check_health(self, err_word: float | None = None):
        """Raise PersistentStepError when a persistent launch's grid barrier timed out:
        its workgroups exited early, so that step's gradient, weights and BN statistics
        are garbage and must neither reach a checkpoint nor keep training.  `err_word`:
        the flag slot (scalars[4]) if the caller has read the scalars already."""
        if self.prn is None:
            return
        if err_word is None:
            bad = bool(self.prn.err.item())
        else:
            bad = err_word != 0.0
        if bad:
            raise PersistentStepError(
                "a persistent-step grid barrier timed out (workgroups not co-resident or lost); "
                f"the step's results are invalid (err={int(self.prn.err.item())})")

    def clear_persist_error(self):
        if self.prn is not None:
            self.prn.err.zero_()

    # ------------------------------------------------------------------ running
    def repack(self):
        """Refresh the bf16 weight copies from the fp32 master (no update)."""
        s = self.sched
        self.nat.sgd_update_pack(self.params.master.data_ptr(), self.grad.data_ptr(),
                                 self.mom.data_ptr(), self.params.n_train, s.init, 0, 0.0, 0.0, [],
                                 [s.init], 0, 0.0, 0.0, 1.0, 0, self.segs.data_ptr(), self.nseg,
                                 self.wbf.data_ptr(), 0, 0, torch.cuda.current_stream().cuda_stream)
        self.nat.ohwi_pack(self.params.master.data_ptr(), self.segs.data_ptr(),
                           self.ohwi_tile0.data_ptr(), self.nseg, self.ohwi_tiles,
                           self.wbf.data_ptr(), 0, torch.cuda.current_stream().cuda_stream)
        if self.stem_s2d:
            self.nat.stem_s2d_pack(self.stem_master, self.stem_w4.data_ptr(),
                                   self.spec.stem.cout, torch.cuda.current_stream().cuda_stream)

    def _run(self, name, stream):
        a, b = self.seg[name]
        self.plan.run(a, b, stream, self.side.cuda_stream, self.comm_stream.cuda_stream)

    def _step_eager(self, need_cost: bool = False):
        st = torch.cuda.current_stream().cuda_stream
        if need_cost:
            self._run("cost", st)
        if self.markers:
            return self._step_marked(st)
        self._run("fwd", st)
        self._run_bwd(st)
        self._run("opt", st)

    def _step_marked(self, st):
        """The eager step inside roctx ranges (DTR_ROCTX=1 / bench --roctx): the
        phases show up as markers in `rocprofv3 --marker-trace` timelines."""
        nvtx = torch.cuda.nvtx   # roctx on ROCm builds of PyTorch
        nvtx.range_push("dtr.step")
        for name, fn in (("fwd", lambda: self._run("fwd", st)), ("bwd+allreduce",
                         lambda: self._run_bwd(st)), ("opt", lambda: self._run("opt", st))):
            nvtx.range_push(f"dtr.{name}")
            fn()
            nvtx.range_pop()
        nvtx.range_pop()

    def _host_allreduce(self, lo, hi):
        """gloo rehearsal: a c10d all-reduce of grad[lo:hi) issued by the host."""
        if self.grad_bf16 is not None:
            buf = self.grad_bf16[lo:hi]
            buf.copy_(self.grad[lo:hi])
            return self.dist.all_reduce_async(buf), lo, hi
        return self.dist.all_reduce_async(self.grad[lo:hi]), lo, hi

    def _host_allreduce_wait(self, works):
        for w, lo, hi in works:
            w.wait()
            if self.grad_bf16 is not None:
                self.grad[lo:hi].copy_(self.grad_bf16[lo:hi])

    def _run_bwd(self, st):
        a, b = self.seg["bwd"]
        side, comm = self.side.cuda_stream, self.comm_stream.cuda_stream
        if self.bucket_sched:
            works, prev = [], a
            for idx, lo, hi in self.bucket_sched:
                if idx > prev:
                    self.plan.run(prev, idx, st, side, comm)
                    prev = idx
                works.append(self._host_allreduce(lo, hi))
            if b > prev:
                self.plan.run(prev, b, st, side, comm)
            self._host_allreduce_wait(works)
        else:
            self.plan.run(a, b, st, self.side.cuda_stream, self.comm_stream.cuda_stream)

    def step_timed(self, need_cost: bool = False) -> dict:
        """One eager step with HIP-event timing per phase (ProfilerHook, bench.py):
        forward, backward compute, the exposed all-reduce tail (from the end of
        the backward's compute to the optimizer's join of the last bucket's
        all-reduce; for gloo rehearsals, the host's c10d waits) and the optimizer."""
        st = torch.cuda.current_stream().cuda_stream
        p = self.plan
        self._steps_run += 1
        if need_cost:
            self._run("cost", st)
            self._cost_at = self._steps_run
        if self.bucket_sched:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
            ev[0].record()
            self._run("fwd", st)
            ev[1].record()
            a, b = self.seg["bwd"]
            works, prev = [], a
            for idx, lo, hi in self.bucket_sched:
                self.plan.run(prev, idx, st, self.side.cuda_stream, self.comm_stream.cuda_stream)
                prev = idx
                works.append(self._host_allreduce(lo, hi))
            self.plan.run(prev, b, st, self.side.cuda_stream, self.comm_stream.cuda_stream)
            ev[2].record()
            self._host_allreduce_wait(works)
            ev[3].record()
            self._run("opt", st)
            ev[4].record()
            torch.cuda.synchronize()
            return {"forward": ev[0].elapsed_time(ev[1]), "backward": ev[1].elapsed_time(ev[2]),
                    "allreduce_exposed": ev[2].elapsed_time(ev[3]),
                    "backward+allreduce": ev[1].elapsed_time(ev[3]),
                    "optimizer": ev[3].elapsed_time(ev[4])}
        p.set_timing(True)
        try:
            self._run("fwd", st)
            self._run_bwd(st)
            self._run("opt", st)
            torch.cuda.synchronize()
        finally:
            p.set_timing(False)
        bwd = p.elapsed_ms(self._t_bwd0, self._t_bwd_done)
        exposed = p.elapsed_ms(self._t_bwd_done, self._t_joined)
        return {"forward": p.elapsed_ms(self._t_fwd0, self._t_bwd0), "backward": bwd,
                "allreduce_exposed": exposed, "backward+allreduce": bwd + exposed,
                "optimizer": p.elapsed_ms(self._t_joined, self._t_opt_end)}

    def comm_info(self) -> dict:
        """How the gradients are exchanged (bench.py JSON)."""
        nat = self.comm is not None
        per = 2 if self.grad_bf16 is not None else 4
        transport = self.comm.transport if nat else ("c10d" if self.bucket_sched else None)
        return {"native_rccl": nat and transport == "rccl",
                "native": nat,
                "transport": transport,
                "fallback_reason": self.comm_fallback_reason,
                "buckets": len(self.buckets) if self.reduce_buckets else 0,
                "allreduce_ops": self._n_allreduce if nat else len(self.bucket_sched),
                "allreduce_bytes": (self._allreduce_bytes if nat else
                                    sum((hi - lo) * per for _, lo, hi in self.bucket_sched)),
                "rccl_library": self.comm.library_path if nat else None,
                "rccl_version": (self.nat.Comm.rccl_version()
                                 if nat and transport == "rccl" else None),
                # the persistent overlap plan's CU budget: CUs left out of the backward
                # grid for the comm stream, and RCCL's channel cap / reported channels
                "overlap_reserve_cus": (self.prn.cus - self.N * self.prn.P - self.prn.wgrad_wgs
                                        if self.persist_overlap else 0),
                **(self.dist.rccl_channel_info() if self.dist is not None else
                   {"rccl_max_nchannels": os.environ.get("NCCL_MAX_NCHANNELS"),
                    "rccl_channels": None}),
                # the communication environment of this run (RCCL / HSA knobs)
                "env": {k: v for k, v in sorted(os.environ.items())
                        if k.startswith(("NCCL_", "RCCL_", "HSA_"))}}

    def capture(self, warmup: int = 2):
        """Run `warmup` real steps on a side stream, then capture one step."""
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._step_eager()
                self._steps_run += 1
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._step_eager()
        self.graph = g
        self._captured = True
        return warmup

    def step(self, need_cost: bool = False):
        """One training step (global_step += 1 on the device).  ``need_cost``: also
        compute 1/2 sum v^2 of this step's (pre-update) weights for the logged cost."""
        if self.graph is not None:
            if need_cost:
                self._run("cost", torch.cuda.current_stream().cuda_stream)
            self.graph.replay()
        else:
            self._step_eager(need_cost)
        self._steps_run += 1
        if need_cost:
            self._cost_at = self._steps_run

    # ------------------------------------------------------------------ io
    def set_batch(self, images, labels):
        """Copy a host/device batch into the static input buffers."""
        if self.input_mode in ("cifar_u8", "imagenet_u8"):
            self.img_u8.copy_(images, non_blocking=True)
        else:
            x = images
            if x.dim() == 4 and tuple(x.shape) != tuple(self.x_in.shape):
                x = self._stem_input(x)
            self.x_in.copy_(x, non_blocking=True)
        self.labels.copy_(labels.to(torch.int32), non_blocking=True)

    def fill_synthetic(self, seed: int = 0):
        g = torch.Generator(device="cpu").manual_seed(seed)
        if self.input_mode in ("cifar_u8", "imagenet_u8"):
            self.img_u8.copy_(torch.randint(0, 256, tuple(self.img_u8.shape), generator=g,
                                            dtype=torch.uint8))
        else:
            npix = self.N * self.spec.image_h * self.spec.image_w
            # s2d: every 16-channel row holds 4 pixels of 3 (+1 zero) channels
            self.nat.synthetic_images(self.x_in.data_ptr(), npix, 3,
                                      4 if self.stem_s2d else self.cpad_in, seed,
                                      torch.cuda.current_stream().cuda_stream)
        self.labels.copy_(torch.randint(0, self.spec.num_classes, (self.N,), generator=g,
                                        dtype=torch.int32))

    def metrics(self, reduce: bool = True) -> dict:
        """Host read of the last step's scalars (synchronises).  The `cost` term
        wd * 1/2 sum v^2 is exact (pre-update weights) when the step ran with
        need_cost=True; otherwise it is computed now from the updated weights.
        ``reduce``: loss and precision over the whole global batch -- a collective
        that EVERY rank must call at the same point; False: this rank's batch."""
        if self._cost_at != self._steps_run:
            self._run("cost", torch.cuda.current_stream().cuda_stream)
            self._cost_at = self._steps_run
        v = self.scalars.detach().cpu().tolist()
        self.check_health(v[4])
        loss_sum, correct, lr, l2 = v[0], v[1], v[2], v[3]
        if reduce and self.dist is not None and self.world > 1:
            t = torch.tensor([loss_sum, correct], device=self.device)
            self.dist.all_reduce_sum(t)
            loss_sum, correct = t.tolist()
            n = self.N * self.world
        else:
            n = self.N
        xent = loss_sum / n
        return {"global_step": int(self.gstep.item()), "cross_entropy": xent,
                "cost": xent + self.wd * l2, "precision": correct / n, "lr": lr, "l2": l2}

    def sync_from_params(self):
        """After loading master/stats from a checkpoint: reset step and repack."""
        self.gstep.fill_(self.params.global_step)
        self.repack()

    def broadcast_parameters(self, src: int = 0):
        """hvd.BroadcastGlobalVariablesHook(0) equivalent: weights, momentum,
        BN moving statistics and global_step from `src` to every rank."""
        if self.dist is None or self.world == 1:
            return
        if self.comm is not None:
            st = torch.cuda.current_stream().cuda_stream
            for t in (self.params.master, self.params.stats, self.mom, self.gstep):
                code = self.nat.COMM_I64 if t.dtype == torch.int64 else self.nat.COMM_F32
                self.comm.broadcast(t.data_ptr(), t.numel(), code, src, st)
        else:
            for t in (self.params.master, self.params.stats, self.mom, self.gstep):
                self.dist.broadcast(t, src)
        self.repack()

    # ------------------------------------------------------------------ eval
    def build_eval_plan(self, batch: int):
        """Forward-only plan in inference mode (BN from moving statistics)."""
        if batch in self.eval_plans:
            return self.eval_plans[batch]
        ev = _EvalPlan(self, batch)
        self.eval_plans[batch] = ev
        return ev


class _EvalPlan:
    """Inference forward (resnet_cifar_main.py:361-421 evaluate()): batch-norm
    with moving statistics, no statistics update, softmax probabilities."""

    def __init__(self, eng: Engine, N: int):
        self.eng = eng
        self.N = N
        nat, spec, dev = eng.nat, eng.spec, eng.device
        H, W = spec.image_h, spec.image_w
        self.img_u8 = torch.zeros((N, 3, H, W), dtype=torch.uint8, device=dev)
        self.x_in = torch.zeros(eng._x_in_shape(N), dtype=BF16, device=dev)
        self.labels = torch.zeros(N, dtype=torch.int32, device=dev)
        self.probs = torch.zeros((N, eng.kpad), device=dev)
        self.xent_ws = torch.empty(eng.nat.softmax_xent_ws_floats(N, eng.kpad), device=dev)
        self.logits = torch.zeros((N, eng.kpad), device=dev)
        self.scalars = torch.zeros(4, device=dev)
        p = nat.Plan()
        self.plan = p
        self.input_plan = nat.Plan()
        if not eng.stem_s2d:   # raw uint8 CIFAR records (run(raw_u8=True))
            self.input_plan.cifar_augment(self.img_u8.data_ptr(), self.x_in.data_ptr(), N, H, W,
                                          eng.cpad_in, 4, 0, 0, 0, 0, 0, 0)
        st = spec.stem
        stem = eng.convs[st.name]
        bufs = []

        def buf(shape):
            t = torch.empty(shape, dtype=BF16, device=dev)
            bufs.append(t)
            return t

        for bn in eng.bns.values():
            p.bn_eval(bn.gamma, bn.beta, bn.mmean, bn.mvar, BN_EPS, bn.spec.channels,
                      bn.scale.data_ptr(), bn.shift.data_ptr())
        y = buf((N, st.ho, st.wo, st.cout))
        p.conv_gemm(0, self.x_in.data_ptr(), stem.ohwi, y.data_ptr(), 0, 0, 0, 0, 0, 0, 0, 0,
                    eng._geom(stem, N), [], [], [], [], [], BN_DECAY, BN_EPS, 1)
        if spec.maxpool:
            ph = _ceil(st.ho, 2)
            pad = max((ph - 1) * 2 + 3 - st.ho, 0) // 2
            z = buf((N, ph, ph, st.cout))
            p.maxpool_fwd(y.data_ptr(), z.data_ptr(), 0,
                          [N, st.ho, st.wo, st.cout, ph, ph, st.cout, 3, 3, 2, pad], 3)
            y = z
        x = y
        for b in spec.blocks:
            bns = [eng.bns[s.name] for s in b.bns]
            convs = [eng.convs[c.name] for c in b.convs]
            res = x
            if b.proj is not None:
                pc = eng.convs[b.proj.name]
                res = buf((N, b.ho, b.wo, b.cout))
                self._conv(p, pc, x, res, bns[0])
            h = x
            for j, c in enumerate(convs):
                last = j == len(convs) - 1
                o = buf((N, c.spec.ho, c.spec.wo, c.spec.cout))
                self._conv(p, c, h, o, bns[j], residual=res if last else None)
                h = o
            x = h
        fbn = eng.bns[spec.final_bn.name]
        F = spec.dense_in
        self.pooled = torch.empty((N, F), dtype=BF16, device=dev)
        p.bnrelu_avgpool(x.data_ptr(), fbn.scale.data_ptr(), fbn.shift.data_ptr(),
                         self.pooled.data_ptr(), N, x.shape[1] * x.shape[2], F)
        p.conv_gemm(0, self.pooled.data_ptr(), eng.dense_ohwi, 0, self.logits.data_ptr(), 0, 0, 0,
                    eng.dense_bias, spec.num_classes, 0, 0, eng._dense_geom(N), [], [], [], [], [], BN_DECAY, BN_EPS, 1)
        sp = self.scalars.data_ptr()
        p.softmax_xent(self.logits.data_ptr(), eng.kpad, self.labels.data_ptr(), N,
                       spec.num_classes, sp, sp + 4, 0, 0, 1.0, self.probs.data_ptr(),
                       self.xent_ws.data_ptr())
        self._bufs = bufs

    def _conv(self, p, c, x, out, pre, residual=None):
        p.conv_gemm(0, x.data_ptr(), c.ohwi, out.data_ptr(), 0,
                    0 if residual is None else residual.data_ptr(), pre.scale.data_ptr(),
                    pre.shift.data_ptr(), 0, 0, 0, 0, self.eng._geom(c, self.N), [], [], [], [], [], BN_DECAY, BN_EPS, 1)

    def run(self, images=None, labels=None, raw_u8: bool = True):
        """Returns (loss_sum, correct, probs[N, classes]) for one eval batch.

        NOTE: shares the per-BN scale/shift buffers with the training plan, so
        it must not run concurrently with a training step (the evaluator runs
        in its own process, like the reference's side-car)."""
        st = torch.cuda.current_stream().cuda_stream
        if images is not None:
            if raw_u8:
                self.img_u8.copy_(images)
                self.input_plan.run(0, self.input_plan.size(), st, 0)
            else:
                x = images.to(self.eng.device)
                if tuple(x.shape) != tuple(self.x_in.shape):
                    x = self.eng._stem_input(x.float())
                self.x_in.copy_(x.to(BF16))
        if labels is not None:
            self.labels.copy_(labels.to(torch.int32))
        self.plan.run(0, self.plan.size(), st, 0)
        v = self.scalars.cpu().tolist()
        return v[0], v[1], self.probs[:, :self.eng.spec.num_classes]
