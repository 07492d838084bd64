#!/usr/bin/env python3
"""Single-process trainer / evaluator (reference resnet_single.py:51-213).

BASELINE config 1: ResNet-20 CIFAR-10 on the CPU, batch 32, synthetic data --
the plumbing path (fp32 PyTorch autograd with TF semantics, no GPU):

    python resnet_single.py --synthetic --train_steps 20

Prints the tfprof-style parameter / FLOP analysis first (resnet_single.py:58-66).
`--log_root` keeps the reference's layout (log_root/train, log_root/eval).
The reference script is broken (HParams fields that do not exist, defect #9);
this one runs.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_tensorflow_resnet_amd.models.spec import build_spec  # noqa: E402
from distributed_tensorflow_resnet_amd.train.driver import main as drive  # noqa: E402
from distributed_tensorflow_resnet_amd.utils.flags import build_parser  # noqa: E402
from distributed_tensorflow_resnet_amd.utils.model_stats import report  # noqa: E402


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    p = build_parser("single")
    p.set_defaults(resnet_size=20, batch_size=32, device="cpu", log_every=10)
    flags, _ = p.parse_known_args(argv)
    defaults = {"--resnet_size": "20", "--batch_size": "32", "--device": "cpu",
                "--log_every": "10"}
    for k, v in defaults.items():
        if not any(a == k or a.startswith(k + "=") for a in argv):
            argv += [f"{k}={v}"]
    if flags.log_root:
        if not any(a.startswith("--train_dir") for a in argv):
            argv.append(f"--train_dir={os.path.join(flags.log_root, 'train')}")
        if not any(a.startswith("--eval_dir") for a in argv):
            argv.append(f"--eval_dir={os.path.join(flags.log_root, 'eval')}")
        if not any(a.startswith("--log_dir") for a in argv):
            argv.append(f"--log_dir={os.path.join(flags.log_root, 'train')}")
    spec = build_spec(flags.dataset, int(dict(a.split("=", 1) for a in argv
                                              if a.startswith("--resnet_size="))["--resnet_size"]))
    print(report(spec, batch=1), flush=True)
    return drive(argv, kind="cifar")


if __name__ == "__main__":
    sys.exit(main())
