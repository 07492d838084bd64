"""Dynamic race check of the native plan by schedule perturbation (GPU).

utils/streamcheck.py certifies the fork/join STRUCTURE of a plan statically, but
it does not know which buffers an op touches (a side-stream read of a buffer the
main stream rewrites after the fork passes it).  No GPU sanitizer runs on this
pool (no XNACK, no GPU ASan), so this module checks the buffers the way a race
shows up in practice -- as a result that depends on the schedule:

1. the reference run: every stream of the plan is folded onto the main stream
   (``Plan.set_perturb(1)``), so the ops execute one at a time in plan order,
   which is a valid sequential schedule of the program;
2. perturbed runs: the real three-stream plan with the per-stream issue
   threads, plus a spinning one-wave delay (csrc/diag.hip) in front of a random
   subset of launches on every stream (``Plan.set_perturb(2, seed, prob,
   max_us)``), a different subset and duration each run and trial, so any pair
   of unordered ops overlaps in a different order each time;
3. the final training state (fp32 master weights, momentum, BN moving
   statistics, global_step) of every perturbed run must equal the reference's
   BIT FOR BIT.  The step is deterministic by construction (fixed-order split-K
   reduce, exact fp64 BN sums, RNG keyed on global_step), so any difference is
   an ordering bug: a missing fork, a missing join, or a buffer reused while an
   unordered stream still reads it.

SURVEY.md §5 "race detection" (stream-ordering asserts and a run-to-run
determinism test).  The reference has no counterpart: TF orders its graph
itself, `/root/reference/resnet_cifar_main.py:328-356`.

  python -m distributed_tensorflow_resnet_amd.utils.racecheck --model cifar_resnet50 \\
      --batch 16 --steps 3 --trials 3
"""
from __future__ import annotations

import argparse
import json
from typing import Callable, Dict, List

import torch


def engine_state(eng) -> Dict[str, torch.Tensor]:
    torch.cuda.synchronize()
    return {"master": eng.params.master.detach().clone(), "momentum": eng.mom.detach().clone(),
            "stats": eng.params.stats.detach().clone(), "global_step": eng.gstep.detach().clone()}


def _diff(ref: Dict[str, torch.Tensor], got: Dict[str, torch.Tensor]) -> List[str]:
    return [k for k in ref if not torch.equal(ref[k], got[k])]


def perturbation_check(make_engine: Callable[[], object], steps: int = 3, trials: int = 3,
                       prob: float = 0.3, max_us: float = 20.0, seed: int = 0) -> dict:
    """Run ``steps`` training steps once serialized and ``trials`` times perturbed,
    each on a fresh engine from ``make_engine()`` (same seeds), and compare the
    final states bitwise.  Returns {"ok", "mismatches": [(trial, [tensors])], ...}."""
    eng = make_engine()
    eng.plan.set_perturb(1)
    for _ in range(steps):
        eng.step()
    ref = engine_state(eng)
    del eng
    mismatches = []
    for t in range(trials):
        eng = make_engine()
        eng.plan.set_perturb(2, seed + 7919 * (t + 1), prob, max_us)
        for _ in range(steps):
            eng.step()
        bad = _diff(ref, engine_state(eng))
        if bad:
            mismatches.append((t, bad))
        del eng
    return {"ok": not mismatches, "mismatches": mismatches, "steps": steps, "trials": trials,
            "prob": prob, "max_us": max_us}


def _make_factory(model: str, batch: int, device, loopback: bool = False,
                  allreduce_dtype: str = "fp32", bucket_mb: float = 0.0):
    """Engine factory; ``loopback``: with the comm stream active -- every bucket
    all-reduced (x2, csrc/comm.h loopback transport) on stream 2 between its
    side-stream producers and the optimizer, bf16 casts included if asked."""
    from .. import native
    from ..models.spec import cifar_spec, imagenet_spec
    from ..train.engine import Engine, cifar_lr_schedule

    if model.startswith("cifar_resnet"):
        spec = cifar_spec(int(model[len("cifar_resnet"):]))
    elif model.startswith("imagenet_resnet"):
        spec = imagenet_spec(int(model[len("imagenet_resnet"):]))
    else:
        raise SystemExit(f"unknown model {model!r}")

    def make():
        kw = {}
        if loopback:
            kw = dict(comm=native().Comm.loopback(2.0), allreduce_dtype=allreduce_dtype,
                      bucket_mb=bucket_mb or None)
        eng = Engine(spec, batch, weight_decay=2e-4, lr_schedule=cifar_lr_schedule(),
                     device=device, seed=7, data_seed=99, use_graph=False, **kw)
        eng.fill_synthetic(3)
        return eng
    return make


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--model", default="cifar_resnet50")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--prob", type=float, default=0.3)
    ap.add_argument("--max_us", type=float, default=20.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--loopback", action="store_true",
                    help="comm stream active: loopback (x2) all-reduce of every bucket")
    ap.add_argument("--allreduce_dtype", default="fp32", choices=("fp32", "bf16"))
    ap.add_argument("--bucket_mb", type=float, default=0.0)
    a = ap.parse_args(argv)
    res = perturbation_check(_make_factory(a.model, a.batch, torch.device("cuda", 0), a.loopback,
                                           a.allreduce_dtype, a.bucket_mb),
                             a.steps, a.trials, a.prob, a.max_us, a.seed)
    print(json.dumps(dict(res, model=a.model, batch=a.batch, loopback=a.loopback,
                          allreduce_dtype=a.allreduce_dtype)))
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    raise SystemExit(main())
