#!/usr/bin/env bash
# Stop the processes a launch/start-*.sh run recorded (reference: stop.sh / stop-2.sh,
# which removed the docker containers).  Usage: launch/stop.sh RUN_DIR
# Kills exactly the recorded process groups (never by name pattern).
set -uo pipefail
RUN_DIR="${1:?usage: stop.sh RUN_DIR}"
shopt -s nullglob
for f in "$RUN_DIR"/*.pid; do
  pid=$(cat "$f")
  if kill -0 "$pid" 2>/dev/null; then
    kill -TERM -- "-$pid" 2>/dev/null || kill -TERM "$pid"
    for _ in $(seq 1 30); do kill -0 "$pid" 2>/dev/null || break; sleep 1; done
    kill -0 "$pid" 2>/dev/null && kill -KILL -- "-$pid" 2>/dev/null
    echo "[stop] $(basename "$f" .pid) ($pid) stopped"
  fi
  rm -f "$f"
done
