#!/bin/bash
# Round 6: PMC passes (bytes, L2 hit, MFMA rate, waits, LDS conflicts) over the ImageNet
# RN50 conv shapes of scripts/roofline.py on the round-6 build (one pass per run).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out && rm -rf gpurun_out/pmc6_a gpurun_out/pmc6_b
A="FETCH_SIZE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
B="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"
ROOFLINE_MANIFEST=gpurun_out/pmc6_manifest.txt timeout -s KILL 240 rocprofv3 --pmc $A --output-format csv \
  -d gpurun_out/pmc6_a -o pmc -- python3 scripts/roofline.py 1 > gpurun_out/pmc6_a.log 2>&1 || exit $?
ROOFLINE_MANIFEST=gpurun_out/pmc6_manifest_b.txt timeout -s KILL 240 rocprofv3 --pmc $B --output-format csv \
  -d gpurun_out/pmc6_b -o pmc -- python3 scripts/roofline.py 1 > gpurun_out/pmc6_b.log 2>&1 || exit $?
find gpurun_out/pmc6_a gpurun_out/pmc6_b -name "*.csv"
