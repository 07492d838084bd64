cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S="128 7 512 512 3 1"
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
P3="FETCH_SIZE WRITE_SIZE"
scripts/gpurun/gpu_steps.sh \
 90 "timeout -s KILL 80 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/pmc7a -- python3 scripts/one_shape.py $S > gpurun_out/pmc7a.log 2>&1" \
 90 "timeout -s KILL 80 rocprofv3 --pmc $P2 --output-format csv -d gpurun_out/pmc7b -- python3 scripts/one_shape.py $S > gpurun_out/pmc7b.log 2>&1" \
 90 "timeout -s KILL 80 rocprofv3 --pmc $P3 --output-format csv -d gpurun_out/pmc7c -- python3 scripts/one_shape.py $S > gpurun_out/pmc7c.log 2>&1" \
 90 "timeout -s KILL 80 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt7 -- python3 scripts/one_shape.py $S > gpurun_out/kt7.log 2>&1"
