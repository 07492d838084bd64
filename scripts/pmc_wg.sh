cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
scripts/gpurun/gpu_steps.sh \
 90 "timeout -s KILL 80 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmcw_a -- python3 scripts/one_shape.py 128 56 64 64 3 1 5 wgrad > gpurun_out/pmcw_a.log 2>&1" \
 90 "timeout -s KILL 80 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmcw_b -- python3 scripts/one_shape.py 128 56 64 64 3 1 5 wgrad > gpurun_out/pmcw_b.log 2>&1" \
 90 "timeout -s KILL 80 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmcw_c -- python3 scripts/one_shape.py 128 7 512 512 3 1 5 wgrad > gpurun_out/pmcw_c.log 2>&1" \
 90 "timeout -s KILL 80 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmcw_d -- python3 scripts/one_shape.py 128 7 512 512 3 1 5 wgrad > gpurun_out/pmcw_d.log 2>&1"
