cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S="128 56 256 64 1 1 5 dgrad,dgrad_bnb"
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
scripts/gpurun/gpu_steps.sh \
 90 "timeout -s KILL 80 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmcb_a -- python3 scripts/one_shape.py $S > gpurun_out/pmcb_a.log 2>&1" \
 90 "timeout -s KILL 80 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmcb_b -- python3 scripts/one_shape.py $S > gpurun_out/pmcb_b.log 2>&1" \
 90 "timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcb_c -- python3 scripts/one_shape.py $S > gpurun_out/pmcb_c.log 2>&1"
