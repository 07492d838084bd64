"""Run a script against another copy of the package (same-box A/B of two native builds):
    python scripts/ab_run.py PKG_PARENT_DIR SCRIPT [args...]
The package is imported from PKG_PARENT_DIR first, so the script's own sys.path insert
finds it already loaded."""
import os
import runpy
import sys

root = os.path.abspath(sys.argv[1])
sys.path.insert(0, root)
import distributed_tensorflow_resnet_amd  # noqa: E402,F401

assert os.path.dirname(os.path.dirname(distributed_tensorflow_resnet_amd.__file__)) == root
sys.argv = sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
