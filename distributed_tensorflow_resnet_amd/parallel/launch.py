"""Local multi-process launcher: one process per GPU (replaces the reference's
docker + ssh + `mpirun -np N -H host:1,...` Horovod launchers and the per-task
PS/worker containers; start-resnet-*-main.sh).

    python -m distributed_tensorflow_resnet_amd.parallel.launch --nproc 8 \
        resnet_cifar_main.py --batch_size 16 --train_dir /tmp/ckpt ...

Sets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT for each child
(env:// rendezvous; torch.distributed "nccl" = RCCL over xGMI).  Failure
handling: if any rank exits non-zero the launcher terminates the others and,
with --max_restarts > 0, relaunches the whole job, which resumes from the
latest complete checkpoint in --train_dir (atomic checkpoint writes).  For
multi-node use torchrun (--nnodes / --rdzv) with the same scripts.
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time


def _spawn(nproc, script, args, port, addr, extra_env):
    procs = []
    for r in range(nproc):
        env = dict(os.environ)
        env.update(extra_env)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(nproc),
                    "LOCAL_WORLD_SIZE": str(nproc), "MASTER_ADDR": addr,
                    "MASTER_PORT": str(port)})
        # dmabuf IPC: the only IPC mode the MI355X hosts support; RCCL's intra-node P2P
        # (xGMI) buffer exchange fails under the legacy mode ("hipIpcGetMemHandle:
        # invalid argument").  An explicit user value wins.
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, script] + list(args), env=env,
                                      start_new_session=True))
    return procs


def _wait(procs, poll_s=0.5):
    """Wait for all ranks; on the first failure terminate the rest. Returns rc."""
    while True:
        alive = False
        for p in procs:
            rc = p.poll()
            if rc is None:
                alive = True
            elif rc != 0:
                for q in procs:
                    if q.poll() is None:
                        try:
                            os.killpg(q.pid, signal.SIGTERM)
                        except ProcessLookupError:
                            pass
                deadline = time.time() + 30
                for q in procs:
                    try:
                        q.wait(timeout=max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        os.killpg(q.pid, signal.SIGKILL)
                return rc
        if not alive:
            return 0
        time.sleep(poll_s)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nproc", "--nproc-per-node", type=int, default=1)
    ap.add_argument("--master_addr", default="127.0.0.1")
    ap.add_argument("--master_port", type=int, default=29512)
    ap.add_argument("--max_restarts", type=int, default=0)
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    rc = 0
    for attempt in range(a.max_restarts + 1):
        extra = {"DTR_RESTART_ATTEMPT": str(attempt)}
        if attempt > 0:
            # fault injection is a one-shot event: do not re-inject on restart
            extra["DTR_FAULT_KILL_STEP"] = "-1"
            print(f"[launch] restarting job (attempt {attempt}) -- ranks resume from the "
                  "latest checkpoint", flush=True)
        procs = _spawn(a.nproc, a.script, a.args, a.master_port + attempt, a.master_addr, extra)
        rc = _wait(procs)
        if rc == 0:
            return 0
        print(f"[launch] a rank failed with exit code {rc}", flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
