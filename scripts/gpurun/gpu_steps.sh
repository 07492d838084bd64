#!/usr/bin/env bash
# Run GPU steps in order, each under its own time limit; stop at the first step
# that faults/aborts/times out (rc not in {0,1}) so nothing else touches the GPU
# after a fault.  Usage: scripts/gpurun/gpu_steps.sh SECONDS "cmd1" SECONDS "cmd2" ...
# Logs go to gpurun_out/step_<n>.log.
set -u
mkdir -p gpurun_out
n=0
while [ $# -ge 2 ]; do
  lim=$1; cmd=$2; shift 2; n=$((n+1))
  log=gpurun_out/step_${n}.log
  echo "=== step $n (limit ${lim}s): $cmd" | tee "$log"
  timeout -k 10 "$lim" bash -c "$cmd" >> "$log" 2>&1
  rc=$?
  echo "=== step $n rc=$rc" | tee -a "$log"
  tail -n 25 "$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping after step $n (rc=$rc)"
    exit $rc
  fi
done
exit 0
