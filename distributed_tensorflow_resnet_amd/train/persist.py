"""Persistent small-batch CIFAR step: descriptor tables + plan ops (csrc/cifar_persist.hip).

At the per-rank batches of the strong-scaling headline config (global batch 128 over
4-8 GPUs = 16-32 images per rank; reference README.md:16-22, resnet_cifar_main.py:326-340)
the launch-per-layer step is a chain of ~110 dependent kernel boundaries.  This path
runs the CIFAR ResNet v2 (resnet_model_official.py:217-278) forward as ONE launch and
its backward as ONE launch: each image is cut into P row slices and one 512-thread
workgroup per slice keeps the slice's activations on-chip across layers (the one halo row
a 3x3 conv needs from each neighbouring slice comes from the tensors the neighbour
publishes anyway), grid barriers only where BatchNorm needs batch statistics (exact fp64
atomic sums), and the CUs beyond the slices compute the weight gradients (fp32 slabs per
image group) while the backward's dgrad chain continues.  The step is then:

    one GPU (5 launches, all on the main stream):
      [augment] -> prn forward -> prn backward -> prn head folds (loss, precision, dense
      gradients: one workgroup) -> sgd_tiles (the weight-gradient slab sums +
      SGD-momentum + both bf16 weight copies, ONE launch)

    world > 1, a native communicator (tune persist_overlap=1, the default): three stage
    buckets (bucket_ranges: stage 3 + final BN + dense, stage 2, stage 1 + stem)
      main:  [augment] -> prn forward -> prn backward (N x P slice workgroups + the
             weight-gradient workgroups; OVERLAP_RESERVE_CUS left out of its grid) ->
             join -> pack(bucket 2) -> all-reduce(bucket 2) -> update(bucket 2, +step)
      comm:  (forked after the forward) head folds -> for buckets 0, 1: a one-wave wait
             for the bucket's count in the backward's barrier region (its weight-gradient
             items + its BatchNorm mark, bucket_target) -> pack (slab sums, bf16 for a
             bf16 exchange: one sgd_tiles launch) -> all-reduce -> update of the bucket's
             parameters, all while the backward still runs on the other CUs
    (persist_overlap=0: pack + ONE all-reduce + ONE update after the backward, main stream.)

Selected by the engine (tune ``persist``: -1 auto = per-rank batch <= AUTO_MAX_BATCH on a supported
CIFAR spec, 0 off, 1 on when supported).
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

PRN_BN = np.dtype([(k, "<u8") for k in ("gamma", "beta", "mmean", "mvar", "mean", "rstd",
                                        "scale", "shift", "dgamma", "dbeta", "acc", "bacc")])
PRN_BLOCK = np.dtype([(k, "<u8") for k in ("x", "h1", "out", "w1f", "w2f", "wpf", "w1b", "w2b",
                                           "wpb", "dout", "dh1", "da2", "da1")] +
                     [(k, "<i4") for k in ("stage", "stride", "bn1", "bn2")])
PRN_ITEM = np.dtype([(k, "<u8") for k in ("dy", "x", "scale", "shift", "part")] +
                    [(k, "<i4") for k in ("kind", "img0", "nimg", "ready", "bucket", "pad_")])
# overlap mode (world > 1): CUs left out of the backward grid for the comm stream's bucket
# waits, packs, RCCL all-reduces and early updates, which run while the backward does (no
# comm-stream kernel fits beside a backward workgroup: each holds a CU's LDS and VGPRs).
# 16 left the stage-3 bucket's pack at 165 us and pushed the chain past the backward's
# end; 48 keeps it inside (world-1 step within 0-7 us of the exchange-after-backward
# plan at bs16-64; 64 / 96 no better: profiles/cifar_comm_overlap.md)
OVERLAP_RESERVE_CUS = 48
# all-reduce buckets of the overlap mode, in the order the backward completes them:
# stage 2 (64 channels) + the final BN + dense, stage 1, stage 0 + the stem
BUCKET_OF_STAGE = (2, 1, 0)

# every supported per-rank batch (MI355X, CIFAR RN50 one-GPU step, round-6 build vs the
# per-layer engine: bs16 0.554-0.556 vs 0.926 ms, bs32 0.565-0.570 vs 0.964, bs64
# 0.638-0.641 vs 1.084, bs128 (1 slice) 0.733-0.743 vs 1.299; profiles/final_check_r06.md)
AUTO_MAX_BATCH = 240


def slices_for(N: int, cus: int, override: int = -1) -> int:
    """Row slices (workgroups) per image of the backward, of the ``cus`` the backward grid
    may fill (the overlap plan's reserve already taken out): 4 while 4N slices leave 32
    CUs for the weight gradients (56 images on 256 CUs), 2 while 2N leave 64 (96
    images), else -- small budgets -- the most slices that leave 16, else 1.  More
    slices shorten each layer, more arrivals lengthen each barrier; with the 64-shard
    arrival counters of round 6 (MI355X, CIFAR RN50 step ms, two runs each;
    forward slicing fixed: bs40 0.594-0.600 at 4 / 0.626-0.632 at 2; bs48 0.607-0.608 /
    0.634; bs56 0.626-0.628 / 0.636-0.638; bs64 0.639-0.641 at 2 / 0.673-0.675 at 1;
    bs80 0.654 / 0.680-0.687; bs96 0.675-0.676 / 0.695-0.701; bs112 0.735-0.737 /
    0.717-0.724).  The engine's tune persist_slices overrides."""
    if override in (1, 2, 4):
        return override
    if 4 * N + 32 <= cus:
        return 4
    if 2 * N + 64 <= cus:
        return 2
    # small CU budgets (a rank on a CU partition, after the overlap reserve): slices
    # before weight-gradient CUs, down to the 16 the check requires (two ranks on CU
    # halves, 16 images per rank: P = 4 with 16 weight-gradient CUs, 1.16 ms/step)
    if N <= 32 and 4 * N + 16 <= cus:
        return 4
    return 2 if N <= 64 and 2 * N + 16 <= cus else 1


def fwd_slices_for(N: int, cus: int, override: int = -1) -> int:
    """Row slices per image of the forward launch.  The forward has no weight-gradient
    workgroups to leave CUs for, and its slicing is independent of the backward's (both
    launches exchange only whole NHWC tensors and global BN sums): 4 while 4N slices fill
    less than 3/4 of the CUs (47 images on 256), 2 while 2N leave 16 (120 images), else 1
    (MI355X, CIFAR RN50 step ms, two runs each, backward slicing fixed: bs40 0.584-0.587
    at 4 / 0.594-0.600 at 2; bs48 0.609-0.610 / 0.607-0.608; bs56 0.643-0.644 /
    0.626-0.628; bs64 0.639-0.641 at 2 / 0.689-0.690 at 1; bs96 0.675-0.676 /
    0.703; bs112 0.719-0.723 / 0.729; bs120 0.730-0.731 / 0.733-0.734; bs128 0.746-0.749
    / 0.740-0.742).  The engine's tune persist_slices overrides."""
    if override in (1, 2, 4):
        return override
    if 16 * N < 3 * cus:
        return 4
    return 2 if 2 * N + 16 <= cus else 1


def check(eng) -> str:
    """'' when the persistent kernels cover this engine's network, batch and device, else
    the reason they do not: the network shape here, every host-side limit of the three
    launches (slices, grids within the CUs, the head folds' LDS) and the co-residency of
    both grids by the occupancy API in one native predicate (prn_check)."""
    spec, nat = eng.spec, eng.nat
    if not spec.dataset.startswith("cifar") or spec.maxpool or eng.stem_s2d:
        return "not a CIFAR network"
    if spec.image_h != 32 or spec.image_w != 32 or spec.dense_in != 64:
        return "not a 32x32 CIFAR ResNet v2"
    st = spec.stem
    if (st.kh, st.kw, st.stride, st.cout) != (3, 3, 1, 16) or st.cin > 8:
        return "stem is not 3x3/1 -> 16"
    nb = len(spec.blocks)
    if nb % 3 or any(b.kind != "building" for b in spec.blocks):
        return "not 3 stages of building blocks"
    n = nb // 3
    for i, b in enumerate(spec.blocks):
        stage = i // n
        if b.cout != 16 << stage or b.ho != 32 >> stage:
            return "stage widths are not 16/32/64"
        first = i % n == 0
        if (b.proj is not None) != first or b.stride != (2 if first and stage else 1):
            return "projection / stride layout is not the CIFAR v2 one"
    cus = nat.cu_count()   # this process's CUs (its CU mask, apply_cu_partition)
    # (at least 16 CUs left for the weight-gradient workgroups, beside the overlap
    # plan's reserve for the comm stream; the backward slices by what is left)
    reserve = OVERLAP_RESERVE_CUS if overlap_planned(eng) else 0
    P = slices_for(eng.N, cus - reserve, eng.persist_slices)
    if eng.N * P + 16 + reserve > cus:
        return (f"{eng.N} x {P} slices + {reserve} reserved CUs leave fewer than 16 of "
                f"{cus} CUs for the weight gradients")
    return str(nat.prn_check(eng.N, P, fwd_slices_for(eng.N, cus, eng.persist_slices), nb,
                             spec.num_classes, eng.kpad))


def overlap_planned(eng) -> bool:
    """Whether the engine takes the overlap plan: a communicator, tune persist_overlap,
    and a backward slicing the OVERLAP_RESERVE_CUS left to the comm stream does not
    reduce.  Where the reserve would cost slices (48 / 56 images on 256 CUs: 4 -> 2; 97 to
    112: 2 -> 1) the buckets go after the backward instead: the world-1 RCCL rehearsal
    over no communicator (`scripts/comm_step_time.py`, round 6) measured overlap / after
    +5.2 / +6.1 us at bs16, +5.3 / +6.3 bs32, +4.4 / +6.5 bs40, +10.1 / +11.4 bs64, but
    +38.9 / +11.0 at bs48 and +18.2 / +7.2 at bs96."""
    if eng.comm is None or not bool(getattr(eng, "persist_overlap_tune", False)):
        return False
    cus = eng.nat.cu_count()
    p = slices_for(eng.N, cus - OVERLAP_RESERVE_CUS, eng.persist_slices)
    # (and the reserved grid still leaves its 16 weight-gradient CUs: a rank on a quarter
    # of the CUs takes the persistent step with the buckets after the backward instead)
    return (p == slices_for(eng.N, cus, eng.persist_slices)
            and eng.N * p + 16 + OVERLAP_RESERVE_CUS <= cus)


def supported(eng) -> bool:
    """Whether the persistent kernels cover this engine's network and batch."""
    return check(eng) == ""


def bucket_ranges(eng):
    """Overlap-mode all-reduce buckets as contiguous ranges of the flat gradient (TF
    variable order: each block's parameters together, the final BN and dense last):
    [(lo, hi, slot names)] in BUCKET_OF_STAGE order -- bucket 0 the last stage's blocks +
    the final BN + dense, bucket 1 the middle stage, bucket 2 the stem + the first stage."""
    spec = eng.spec
    nps = len(spec.blocks) // 3
    stage_of = {spec.stem.name: 0, spec.final_bn.name: 2, "dense": 2}
    for i, b in enumerate(spec.blocks):
        for layer in list(b.convs) + list(b.bns) + ([b.proj] if b.proj is not None else []):
            stage_of[layer.name] = i // nps
    out = [[None, None, []] for _ in BUCKET_OF_STAGE]
    for s in eng.params.train_slots:
        r = out[BUCKET_OF_STAGE[stage_of[s.name.rsplit("/", 1)[0]]]]
        r[0] = s.offset if r[0] is None else min(r[0], s.offset)
        r[1] = s.offset + s.numel if r[1] is None else max(r[1], s.offset + s.numel)
        r[2].append(s.name)
    for lo, hi, names in out:   # contiguous: the slots of a bucket tile [lo, hi)
        assert sum(sl.numel for sl in eng.params.train_slots if sl.name in set(names)) == hi - lo
    return [tuple(r) for r in out]


def fault_injection_bar(rank: int) -> int:
    """Tests only: the forward grid barrier at which workgroup 0 abandons its launch
    (DTR_PRN_FAULT_BAR = ``bar`` on every rank or ``bar@rank`` on one rank of the job: a
    lost workgroup), -1 off.  Honoured only with DTR_TEST_FAULTS=1."""
    spec = os.environ.get("DTR_PRN_FAULT_BAR", "-1")
    bar, _, only = spec.partition("@")
    if int(bar) < 0 or os.environ.get("DTR_TEST_FAULTS", "0") != "1":
        return -1
    return int(bar) if only == "" or int(only) == rank else -1


def _stage(b) -> int:
    return int(math.log2(b.cout // 16))


class PersistStep:
    """Device tables and buffers of the persistent step for one Engine."""

    def __init__(self, eng):
        self.eng = eng
        nat, spec, N, dev = eng.nat, eng.spec, eng.N, eng.device
        sizes = nat.prn_struct_bytes()
        assert sizes == [PRN_BN.itemsize, PRN_BLOCK.itemsize, PRN_ITEM.itemsize], sizes
        blocks = spec.blocks
        nb = len(blocks)
        self.nblocks = nb
        # BatchNorm table: block i's two BNs at 2i, 2i + 1, the final BN last
        order = [bn for b in blocks for bn in b.bns] + [spec.final_bn]
        bn_rows = np.zeros(len(order), dtype=PRN_BN)
        for r, bs in zip(bn_rows, order):
            e = eng.bns[bs.name]
            r["gamma"], r["beta"], r["mmean"], r["mvar"] = e.gamma, e.beta, e.mmean, e.mvar
            r["mean"], r["rstd"] = e.mean.data_ptr(), e.rstd.data_ptr()
            r["scale"], r["shift"] = e.scale.data_ptr(), e.shift.data_ptr()
            r["dgamma"], r["dbeta"] = e.dgamma, e.dbeta
            r["acc"], r["bacc"] = e.acc.data_ptr(), e.bacc.data_ptr()
        self.bn_dev = self._dev(bn_rows)
        self.cus = nat.cu_count()   # this process's CUs (its CU mask)
        self.overlap = bool(getattr(eng, "persist_overlap", False))
        # the backward grid leaves the overlap plan's reserve to the comm stream
        self.P = slices_for(N, self.cus - (OVERLAP_RESERVE_CUS if self.overlap else 0),
                            eng.persist_slices)                       # backward
        self.P_fwd = fwd_slices_for(N, self.cus, eng.persist_slices)  # forward
        # barrier-timeout flag: slot 4 of the engine's scalars, so the host read of the
        # logged metrics (Engine.metrics) sees it at no extra cost; never cleared by the
        # kernels (Engine.clear_persist_error)
        self.err = eng.scalars[4:5].view(torch.int32)
        self.fault_bar = fault_injection_bar(eng.dist.rank if eng.dist is not None else 0)
        self.dpool = torch.zeros((N, 64), device=dev)
        self.dx0 = torch.empty_like(eng.X[0])
        # per-block backward gradients published to the weight-gradient workgroups
        self.dout = [torch.empty_like(eng.X[i + 1]) for i in range(nb)]
        self.dh1 = [torch.empty_like(eng.H1[i]) for i in range(nb)]
        # dgrad outputs before their BN backward: the neighbouring slices recompute their
        # halo rows of the BN-backward output from these (no neighbours at 1 slice)
        none = torch.empty(0, dtype=eng.X[0].dtype, device=dev)
        self.da2 = [torch.empty_like(eng.H1[i]) if self.P > 1 else none for i in range(nb)]
        self.da1 = [torch.empty_like(eng.X[i]) if self.P > 1 else none for i in range(nb)]
        rows = np.zeros(nb, dtype=PRN_BLOCK)
        for i, (r, b) in enumerate(zip(rows, blocks)):
            c1, c2 = eng.convs[b.convs[0].name], eng.convs[b.convs[1].name]
            r["x"], r["h1"], r["out"] = (eng.X[i].data_ptr(), eng.H1[i].data_ptr(),
                                         eng.X[i + 1].data_ptr())
            r["w1f"], r["w2f"], r["w1b"], r["w2b"] = c1.ohwi, c2.ohwi, c1.hwio, c2.hwio
            if b.proj is not None:
                cp = eng.convs[b.proj.name]
                r["wpf"], r["wpb"] = cp.ohwi, cp.hwio
            r["dout"], r["dh1"] = self.dout[i].data_ptr(), self.dh1[i].data_ptr()
            r["da2"], r["da1"] = self.da2[i].data_ptr(), self.da1[i].data_ptr()
            r["stage"], r["stride"] = _stage(b), b.stride
            r["bn1"], r["bn2"] = 2 * i, 2 * i + 1
        self.block_dev = self._dev(rows)
        self._build_items()

    def _dev(self, arr):
        return torch.from_numpy(arr.view(np.uint8).copy()).to(self.eng.device)

    def _build_items(self):
        """Weight-gradient work items in the order the backward publishes their dy
        (`ready` = backward barrier count after which it is visible; barrier 1 is the
        final BN): per block j (last block first) conv2 and the projection with the
        block's dout (stored after the block's first arrive) at 2j + 3, conv1 with dh1
        (stored after the second) at 2j + 4; the stem after the final arrive (2nb + 2).
        Images are grouped per item (the grouped reduce sums one slab per group): a
        quarter of the batch for stages 2-3, whose items have the rest of the backward
        to run in; 4 images for stage 1 and the stem, whose items only become ready at
        the end of the backward -- their duration is the launch's tail (bs128: 32-image
        items left ~140 us of tail after the last slice finished); the convs released
        last (the stem, the first block's, the second block's conv1) at N / 64 images,
        one image up to bs64 (bs16 / bs32 steps 1.3-2.4 % faster than 4-image items; bs128
        at 2 instead of 4 images 0.734 -> 0.731 ms, three same-box rounds; at most 64 slabs
        per conv for the optimizer to sum)."""
        eng, spec, N = self.eng, self.eng.spec, self.eng.N
        nat = eng.nat
        blocks = spec.blocks
        nb = len(blocks)

        tail_ready = 2 * nb   # the last block's convs, the stem, the block before's conv1

        def groups_of(name):
            c = eng.convs[name]
            size = 4 if c.spec.cout == 16 else max(1, math.ceil(N / 4))
            if ready_of[name] >= tail_ready:
                size = max(1, math.ceil(N / 64))
            return [(g0, min(size, N - g0)) for g0 in range(0, N, size)]
        convs = []   # (name, dy, x, bn scale, bn shift, ready, stage)
        for j, i in enumerate(range(nb - 1, -1, -1)):
            b = blocks[i]
            bn1, bn2 = eng.bns[b.bns[0].name], eng.bns[b.bns[1].name]
            d_out, d_h1 = self.dout[i].data_ptr(), self.dh1[i].data_ptr()
            st = _stage(b)
            convs.append((b.convs[1].name, d_out, eng.H1[i].data_ptr(), bn2, 2 * j + 3, st))
            if b.proj is not None:
                convs.append((b.proj.name, d_out, eng.X[i].data_ptr(), bn1, 2 * j + 3, st))
            convs.append((b.convs[0].name, d_h1, eng.X[i].data_ptr(), bn1, 2 * j + 4, st))
        convs.append((spec.stem.name, self.dx0.data_ptr(), eng.x_in.data_ptr(), None, 2 * nb + 2, 0))
        ready_of = {name: ready for name, _, _, _, ready, _ in convs}
        tot = 0
        self.part_off, self.splits = {}, {}
        for name, *_ in convs:
            c = eng.convs[name]
            s = c.spec
            self.part_off[name] = tot
            self.splits[name] = len(groups_of(name))
            tot += self.splits[name] * s.cout * s.kh * s.kw * c.cin
        self.part = torch.empty(max(tot, 1), device=eng.device)
        items = []
        self.stage_of = {name: st for name, *_, st in convs}
        self.bucket_items = [0] * len(BUCKET_OF_STAGE)
        for name, dy, x, bn, ready, st in convs:
            c = eng.convs[name]
            s = c.spec
            kind = nat.prn_item_kind(c.cin, s.cout, s.kh, s.stride)
            assert kind >= 0, (name, c.cin, s.cout, s.kh, s.stride)
            slab = s.cout * s.kh * s.kw * c.cin
            for gi, (g0, gn) in enumerate(groups_of(name)):
                r = np.zeros(1, dtype=PRN_ITEM)[0]
                r["dy"], r["x"] = dy, x
                if bn is not None:
                    r["scale"], r["shift"] = bn.scale.data_ptr(), bn.shift.data_ptr()
                r["part"] = self.part.data_ptr() + 4 * (self.part_off[name] + gi * slab)
                r["kind"], r["img0"], r["nimg"], r["ready"] = kind, g0, gn, ready
                r["bucket"] = BUCKET_OF_STAGE[st] if self.overlap else -1
                if self.overlap:
                    self.bucket_items[BUCKET_OF_STAGE[st]] += 1
                items.append(r)
        self.items = np.array(items, dtype=PRN_ITEM)
        self.item_dev = self._dev(self.items)
        reserve = OVERLAP_RESERVE_CUS if self.overlap else 0
        self.wgrad_wgs = max(1, min(self.cus - N * self.P - reserve, len(items)))
        self.convs = [c[0] for c in convs]

    def bucket_target(self, b: int) -> int:
        """Count bucket b's line reaches when its gradients are complete (overlap mode):
        one per weight-gradient item of its convs + slice workgroup 0's BatchNorm mark."""
        return self.bucket_items[b] + 1

    def pending(self):
        """_pending entries (grouped-reduce descriptors) of every conv's slabs."""
        eng = self.eng
        out = {}
        for name in self.convs:
            c = eng.convs[name]
            s = c.spec
            out[c.name] = (self.part.data_ptr() + 4 * self.part_off[name], c.grad, self.splits[name],
                           s.cout, s.cout, s.kh * s.kw, c.cin, c.cin_valid)
        return out

    def args(self, pool_ptr: int, bar_ptr: int, bn_decay: float, bn_eps: float,
             fwd: bool = False):
        """Plan-op arguments of the forward (fwd) or backward launch."""
        eng, spec = self.eng, self.eng.spec
        ptrs = [self.block_dev.data_ptr(), self.bn_dev.data_ptr(), eng.x_in.data_ptr(),
                eng.convs[spec.stem.name].ohwi, pool_ptr,
                bar_ptr, self.err.data_ptr(), eng.dense_hwio, eng.dense_bias,
                eng.labels.data_ptr(), eng.pooled.data_ptr(), eng.dlogits.data_ptr(),
                eng.xent_ws.data_ptr(), self.dpool.data_ptr(), self.dx0.data_ptr(),
                self.item_dev.data_ptr()]
        # backward / head-fold launches: the head's batch folds' outputs (loss, precision,
        # dense bias and weight gradients; prn_head)
        sp = eng.scalars.data_ptr()
        ptrs += [0, 0, 0, 0] if fwd else [sp, sp + 4, eng.dense_bias_grad, eng.dense_grad]
        ints = [self.nblocks, len(self.items), eng.N, self.P_fwd if fwd else self.P,
                spec.num_classes, eng.kpad, 1,
                self.wgrad_wgs, self.fault_bar if fwd else -1, int(self.overlap and not fwd)]
        ints += list(BUCKET_OF_STAGE) if self.overlap else [-1, -1, -1]
        floats = [1.0 / eng.global_batch, bn_decay, bn_eps]
        return ptrs, ints, floats
