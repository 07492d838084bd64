#!/bin/bash
# Round 3: PMC passes (bytes, L2 hit, MFMA rate, waits) over the ImageNet RN50 conv shapes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
A="FETCH_SIZE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
B="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"
ROOFLINE_MANIFEST=gpurun_out/pmc_manifest.txt timeout -s KILL 240 rocprofv3 --pmc $A --output-format csv \
  -d gpurun_out/pmc_a -o pmc -- python3 scripts/roofline.py 1 > gpurun_out/pmc_a.log 2>&1 || exit $?
ROOFLINE_MANIFEST=gpurun_out/pmc_manifest_b.txt timeout -s KILL 240 rocprofv3 --pmc $B --output-format csv \
  -d gpurun_out/pmc_b -o pmc -- python3 scripts/roofline.py 1 > gpurun_out/pmc_b.log 2>&1 || exit $?
find gpurun_out/pmc_a gpurun_out/pmc_b -name "*.csv" | head
