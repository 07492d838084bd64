"""Command-line flags with the reference's names and defaults.

The reference defines ~25 `tf.app.flags` per entrypoint (resnet_cifar_main.py:
34-97, resnet_imagenet_main.py:33-104, resnet_model.py:30, the *_eval.py
scripts).  One argparse builder reproduces them all -- same spelling, same
defaults per entrypoint -- and accepts absl's boolean spellings (`--flag`,
`--noflag`, `--flag=true|false`).  New flags for this framework:

  --resnet_size      (reference hard-codes 50, resnet_model.py:72,74 -- defect #8)
  --dtype            bf16 (GPU compute) | fp32 (CPU path)
  --synthetic        synthetic data of the dataset's shape
  --bucket_mb        gradient all-reduce bucket size
  --device           auto | gpu | cpu
  --use_graph        capture the training step in a hipGraph
  --seed, --log_every, --save_checkpoint_steps/_secs, --profile_steps, ...
"""
from __future__ import annotations

import argparse
import sys

VARIABLE_UPDATES = ("parameter_server", "replicated", "distributed_replicated", "independent",
                    "distributed_all_reduce", "collective_all_reduce", "horovod")

_DEFAULTS = {
    # name: (cifar, imagenet)
    "dataset": ("cifar10", "imagenet"),
    "train_data_path": ("/home/hdd0/dataset/cifar10_data", ""),
    "train_steps": (2000, 200),
    "batch_size": (32, 128),
    "resnet_size": (50, 50),
    "log_every": (20, 40),            # LoggingTensorHook every_n_iter
    "weight_decay": (2e-4, 1e-4),     # _WEIGHT_DECAY (resnet_cifar_main.py:112) / :472
}


def str2bool(v) -> bool:
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in ("1", "true", "t", "yes", "y"):
        return True
    if s in ("0", "false", "f", "no", "n"):
        return False
    raise argparse.ArgumentTypeError(f"not a boolean: {v!r}")


def _absl_bools(argv, bool_names):
    """Translate absl `--noflag` / bare `--flag` spellings for boolean flags."""
    out = []
    for a in argv:
        if a.startswith("--no") and a[4:] in bool_names:
            out.append(f"--{a[4:]}=false")
        elif a.startswith("--") and "=" not in a and a[2:] in bool_names:
            out.append(f"--{a[2:]}=true")
        else:
            out.append(a)
    return out


class FlagParser(argparse.ArgumentParser):
    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self._bools = set()

    def add_bool(self, name, default, help_):
        self._bools.add(name)
        self.add_argument(f"--{name}", type=str2bool, default=default, nargs="?", const=True,
                          help=help_)

    def parse_args(self, args=None, namespace=None):
        argv = sys.argv[1:] if args is None else list(args)
        return super().parse_args(_absl_bools(argv, self._bools), namespace)

    def parse_known_args(self, args=None, namespace=None):
        argv = sys.argv[1:] if args is None else list(args)
        return super().parse_known_args(_absl_bools(argv, self._bools), namespace)


def build_parser(kind: str = "cifar", description: str | None = None) -> FlagParser:
    """kind: cifar | imagenet (train entrypoints), cifar_eval | imagenet_eval, single."""
    im = 1 if kind.startswith("imagenet") else 0
    p = FlagParser(description=description, allow_abbrev=False)
    d = {k: v[im] for k, v in _DEFAULTS.items()}
    is_eval = kind.endswith("_eval")
    # ---- reference flags (resnet_cifar_main.py:34-97 / resnet_imagenet_main.py:33-104)
    p.add_argument("--dataset", default=d["dataset"], help="cifar10, cifar100 or imagenet")
    p.add_argument("--mode", default="eval" if is_eval else "train",
                   help="train | eval | train_and_eval")
    p.add_argument("--train_data_path", default=d["train_data_path"],
                   help="Filepattern/dir for training data.")
    p.add_argument("--eval_data_path", default="", help="Filepattern/dir for eval data")
    p.add_argument("--image_size", type=int, default=32, help="Image side length (declared, unused).")
    p.add_argument("--train_dir", default="", help="Directory to keep training outputs (checkpoints).")
    p.add_argument("--eval_dir", default="", help="Directory to keep eval outputs.")
    p.add_argument("--eval_batch_count", type=int, default=50, help="Number of batches to eval.")
    p.add_bool("eval_once", False, "Whether evaluate the model only once.")
    p.add_argument("--log_dir", default="", help="Directory for training summaries.")
    p.add_argument("--log_root", default="", help="Legacy root dir (resnet_single/eval scripts).")
    p.add_argument("--num_gpus", type=int, default=0,
                   help="GPUs per worker (reference: gpu = task_index %% num_gpus).")
    p.add_argument("--task_index", type=int, default=None, help="Worker index (PS mode).")
    p.add_argument("--replicas_to_aggregate", type=int, default=None,
                   help="Gradients to aggregate per step (PS sync mode).")
    p.add_argument("--train_steps", type=int, default=d["train_steps"],
                   help="Number of (global) training steps to perform.")
    p.add_argument("--num_epochs", type=int, default=90 if im else 1000, help="Dataset repeats.")
    p.add_argument("--batch_size", type=int, default=d["batch_size"], help="Per-process batch size.")
    p.add_argument("--learning_rate", type=float, default=0.01,
                   help="Declared, unused by ResNet (the LR schedule hook sets it).")
    p.add_argument("--_FILE_SHUFFLE_BUFFER", type=float, default=1024)
    p.add_argument("--_SHUFFLE_BUFFER", type=float, default=1024)
    p.add_bool("sync_replicas", True, "Synchronous replicas (always true here: sync DP).")
    p.add_bool("existing_servers", False, "Use existing servers (PS mode; ignored).")
    p.add_argument("--ps_hosts", default="localhost:2222", help="PS hosts (ignored: no PS).")
    p.add_argument("--worker_hosts", default="localhost:2223,localhost:2224",
                   help="Worker hosts; for multi-node runs use MASTER_ADDR/torchrun instead.")
    p.add_argument("--job_name", default=None, help="worker | ps")
    p.add_argument("--data_format", default="channels_first",
                   help="Accepted for compatibility; kernels are always NHWC.")
    p.add_argument("--num_intra_threads", type=int, default=0)
    p.add_argument("--num_inter_threads", type=int, default=0)
    p.add_argument("--variable_update", default="parameter_server", choices=VARIABLE_UPDATES,
                   help="All synchronous modes map to RCCL all-reduce data parallelism; "
                        "'independent' trains ranks without gradient exchange.")
    p.add_bool("use_horovod", False, "Accepted for compatibility (all-reduce is always on).")
    p.add_argument("--num_parallel_calls", type=int, default=5, help="Input pipeline workers.")
    # ---- new flags
    p.add_argument("--resnet_size", type=int, default=d["resnet_size"])
    p.add_argument("--num_classes", type=int, default=None)
    p.add_argument("--device", default="auto", choices=("auto", "gpu", "cpu"))
    p.add_argument("--dtype", default="bf16", choices=("bf16", "fp32"))
    p.add_bool("synthetic", False, "Synthetic data of the dataset's shape.")
    p.add_argument("--weight_decay", type=float, default=d["weight_decay"])
    p.add_argument("--optimizer", default="mom", choices=("mom", "sgd"))
    p.add_argument("--bucket_mb", type=float, default=0.0,
                   help="All-reduce bucket size (MiB); 0 = auto (~4 buckets, <= 25 MiB).")
    p.add_bool("use_graph", False, "Capture the training step in a hipGraph (single stream; "
               "default eager native plan with a second weight-gradient stream).")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--log_every", type=int, default=d["log_every"])
    p.add_argument("--summary_every", type=int, default=100)
    p.add_argument("--save_checkpoint_steps", type=int, default=1000)
    p.add_argument("--save_checkpoint_secs", type=float, default=0.0,
                   help="If > 0, checkpoint every N seconds (Horovod path used 60).")
    p.add_argument("--max_to_keep", type=int, default=5)
    p.add_argument("--eval_interval_secs", type=float, default=60.0)
    p.add_argument("--eval_batch_size", type=int, default=100)
    p.add_argument("--profile_steps", default="", help="e.g. '50:60' -> per-phase timing report")
    p.add_bool("check_numerics", False, "Abort on NaN/Inf loss (tf.check_numerics analogue).")
    p.add_argument("--fault_kill_step", type=int, default=-1,
                   help="Fault injection: rank --fault_kill_rank exits at this step.")
    p.add_argument("--fault_kill_rank", type=int, default=0)
    p.add_bool("reset_persist_fault", False,
               "Delete the persist_fault marker in --train_dir (left by an attempt whose "
               "persistent CIFAR step failed a grid barrier) so this attempt selects the "
               "persistent step again.")
    p.add_argument("--step_watchdog_secs", type=float, default=0.0,
                   help="If > 0, abort (exit 3, for the launcher to restart from the latest "
                        "checkpoint) when no step completes for this many seconds.  Multi-rank "
                        "jobs always run the watchdog (limit --comm_timeout_secs when this is 0), "
                        "which also polls the native communicator's async error.")
    p.add_argument("--comm_timeout_secs", type=float, default=600.0,
                   help="Collective timeout: the process group's, the native communicator's "
                        "init / shm waits, and the multi-rank step watchdog's default limit "
                        "(on expiry: ncclCommAbort, exit 3).")
    p.add_argument("--lr_schedule_scale", type=float, default=1.0,
                   help="Multiply the LR schedule's step boundaries (and warm-up) by this "
                        "factor: compressed schedules for short runs (convergence tests).")
    p.add_argument("--lr_value_scale", type=float, default=1.0,
                   help="Multiply every LR value of the schedule (and its warm-up) by this "
                        "factor: the linear scaling rule when the global batch differs from "
                        "the reference's (ImageNet: 0.4 for 8 x 128 images).")
    p.add_argument("--allreduce_dtype", default="fp32", choices=("fp32", "bf16"),
                   help="Gradient all-reduce precision: bf16 halves the bytes on xGMI (fp32 "
                        "master weights and optimizer are unchanged).")
    return p


def warn_unsupported(flags, log) -> None:
    """Flags the MI355X framework accepts but does not act on (PS/gRPC topology)."""
    if flags.variable_update == "parameter_server" and flags.job_name:
        log(f"[flags] --variable_update=parameter_server --job_name={flags.job_name}: parameter "
            "servers are not rebuilt; running synchronous RCCL data parallelism instead.")
        if flags.job_name == "ps":
            log("[flags] this process was started as a PS task and has nothing to do; exiting.")
    if not flags.sync_replicas:
        log("[flags] --sync_replicas=False (async PS) is not supported; training synchronously.")
