#!/bin/bash
# Round-6 PMC tables of the persistent CIFAR step (round-6 kernels: 64 shards, new slicing): bs16 (4 slices), bs32 (4)
# and bs128 (1 slice).  Four counter passes per configuration (rocprofv3 does not split
# counters over passes); scripts/pmc_merge.py joins them.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
B="SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS"
mkdir -p gpurun_out/pmc6c
for cfg in "p16:16" "p32:32" "p128:128"; do
  IFS=: read tag b <<< "$cfg"
  i=0
  for set in "$A" "$B" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc6c/$tag-$i -- python3 bench.py --batch $b --steps 6 --warmup 3 --phase-steps 0 > gpurun_out/pmc6c/$tag-$i.log 2>&1 || { tail -5 gpurun_out/pmc6c/$tag-$i.log; exit 1; }
  done
  echo "$tag done"
done
