#!/bin/bash
# Round 5: early weight prefetch, wave-0 drains at P=1 -- pins, then the previous build
# (ab_old/) vs this one, same box, alternating runs; then the LDS conflict counter.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread \
  tests/test_persist_gpu.py tests/test_golden_gpu.py > gpurun_out/r5l_tests.log 2>&1 || { tail -60 gpurun_out/r5l_tests.log; exit 1; }
tail -1 gpurun_out/r5l_tests.log
for r in 1 2; do
  for b in 128 32 16; do
    for v in old new; do
      if [ $v = old ]; then cmd="python scripts/ab_run.py ab_old bench.py"; else cmd="python bench.py"; fi
      timeout -k 10 200 $cmd --batch $b --steps 300 --warmup 30 > gpurun_out/r5l_${v}_b$b.json 2> gpurun_out/r5l_err.log || { tail -20 gpurun_out/r5l_err.log; exit 1; }
      echo "round $r bs$b $v $(python -c "import json;d=json.load(open('gpurun_out/r5l_${v}_b$b.json'));print(d['ms_per_step'])")"
    done
  done
done
B="SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS"
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
mkdir -p gpurun_out/pmc5l
for b in 128 16; do
  i=0
  for set in "$A" "$B"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc5l/p$b-$i -- python3 bench.py --batch $b --steps 6 --warmup 3 --phase-steps 0 > gpurun_out/pmc5l/p$b-$i.log 2>&1 || { tail -5 gpurun_out/pmc5l/p$b-$i.log; exit 1; }
  done
done
echo pmc done
