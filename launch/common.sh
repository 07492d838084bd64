#!/usr/bin/env bash
# Shared helpers for the launch/ scripts (MI355X equivalents of the reference's
# docker / mpirun / SLURM launchers).  One process per GPU through
# the package launcher (RANK/LOCAL_RANK/WORLD_SIZE env rendezvous, RCCL over xGMI),
# restart-on-failure with resume from the latest checkpoint, PID files for stop.sh.
set -euo pipefail
REPO="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
PY="${PYTHON:-python3}"
# dmabuf IPC: the only IPC mode the MI355X hosts support -- under the legacy mode RCCL's
# intra-node P2P (xGMI) buffer exchange fails with "hipIpcGetMemHandle: invalid argument"
export HSA_ENABLE_IPC_MODE_LEGACY="${HSA_ENABLE_IPC_MODE_LEGACY:-0}"
export MASTER_ADDR="${MASTER_ADDR:-127.0.0.1}"

# run_bg NAME LOGFILE CMD... : start CMD in its own process group, record the PID
run_bg() {
  local name=$1 log=$2
  shift 2
  mkdir -p "$RUN_DIR" "$(dirname "$log")"
  setsid "$@" >"$log" 2>&1 < /dev/null &
  echo $! >"$RUN_DIR/$name.pid"
  echo "[launch] $name pid $! -> $log"
}
