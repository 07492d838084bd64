#!/bin/bash
# Round-4 PMC tables: the persistent CIFAR step at bs16 (4 slices) and bs128 (1 slice), and
# the launch-per-layer bs128 step (direct convs, weight gradients).  Four counter passes per
# configuration (rocprofv3 does not split counters over passes).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
B="SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS"
mkdir -p gpurun_out/pmc2
for cfg in "p16:persist=1:16" "p128:persist=1:128" "l128:persist=0:128"; do
  IFS=: read tag tune b <<< "$cfg"
  i=0
  for set in "$A" "$B" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    DTR_TUNE=$tune timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc2/$tag-$i -- python3 bench.py --batch $b --steps 6 --warmup 3 --phase-steps 0 > gpurun_out/pmc2/$tag-$i.log 2>&1 || { tail -5 gpurun_out/pmc2/$tag-$i.log; exit 1; }
  done
  echo "$tag done"
done
