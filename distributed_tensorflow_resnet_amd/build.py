"""Build the native extension ``_C`` in-tree with hipcc for gfx950.

No torch.utils.cpp_extension (which would hipify sources): every ``csrc/*.hip``
file is compiled directly with ``hipcc --offload-arch=gfx950`` and the pybind11
bindings + executor (``csrc/bindings.cpp``) are compiled with hipcc as host code.
The shared object links the HIP runtime by soname ``libamdhip64.so.7``; at import
time torch has already loaded its own copy of that soname, so one runtime is
shared by torch and the extension.

Usage:  python -m distributed_tensorflow_resnet_amd.build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(PKG_DIR, "csrc", "build")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
OUT = os.path.join(PKG_DIR, "_C" + EXT_SUFFIX)
ARCH = os.environ.get("DTR_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

COMMON_FLAGS = [
    "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
    "-Wno-unused-result", "-Wno-unused-variable",
]


# per-file extra flags (none at present; e.g. ["-mllvm", "-amdgpu-mfma-vgpr-form=1"] keeps
# a one-wave-per-SIMD kernel's MFMA accumulators in arch VGPRs, profiles/imagenet_wide.md)
FILE_FLAGS: dict = {}


def _sources():
    """Device code (*.hip), host-only C++ (*.cpp except the bindings), bindings."""
    hips = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))
    hosts = sorted(f for f in os.listdir(CSRC) if f.endswith(".cpp") and f != "bindings.cpp")
    return ([os.path.join(CSRC, f) for f in hips] + [os.path.join(CSRC, f) for f in hosts],
            os.path.join(CSRC, "bindings.cpp"))


def _headers_digest() -> str:
    h = hashlib.sha1()
    for f in sorted(os.listdir(CSRC)):
        if f.endswith(".h"):
            with open(os.path.join(CSRC, f), "rb") as fh:
                h.update(fh.read())
    h.update(" ".join(COMMON_FLAGS).encode())
    return h.hexdigest()


def _file_digest(path: str, extra: str) -> str:
    h = hashlib.sha1(extra.encode())
    with open(path, "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()


def _compile(src: str, obj: str, flags: list[str]) -> None:
    cmd = [HIPCC] + flags + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> str:
    """Compile (incrementally) and link ``_C``; returns the .so path."""
    os.makedirs(BUILD_DIR, exist_ok=True)
    hips, binding = _sources()
    hdr = _headers_digest()
    import pybind11

    py_inc = sysconfig.get_paths()["include"]
    bind_flags = COMMON_FLAGS + [f"-I{pybind11.get_include()}", f"-I{py_inc}", "-fvisibility=hidden"]
    todo = []
    objs = []
    for src in hips + [binding]:
        flags = bind_flags if src == binding else COMMON_FLAGS
        flags = flags + FILE_FLAGS.get(os.path.basename(src), [])
        digest = _file_digest(src, hdr + " ".join(flags))
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
        stamp = obj + ".sha1"
        objs.append(obj)
        fresh = (not force and os.path.exists(obj) and os.path.exists(stamp)
                 and open(stamp).read() == digest)
        if not fresh:
            todo.append((src, obj, flags, stamp, digest))
    if todo:
        jobs = jobs or min(len(todo), max(1, (os.cpu_count() or 4)), 16)
        if verbose:
            print(f"[dtr build] compiling {len(todo)} unit(s) for {ARCH} with {jobs} job(s)", flush=True)
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = {ex.submit(_compile, s, o, f): (s, o, st, d) for s, o, f, st, d in todo}
            for fut in cf.as_completed(futs):
                s, o, st, d = futs[fut]
                fut.result()
                with open(st, "w") as fh:
                    fh.write(d)
    need_link = bool(todo) or not os.path.exists(OUT) or any(
        os.path.getmtime(o) > os.path.getmtime(OUT) for o in objs)
    if need_link:
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", OUT] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"[dtr build] linked {OUT}", flush=True)
    return OUT


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs)
    return 0


if __name__ == "__main__":
    sys.exit(main())
