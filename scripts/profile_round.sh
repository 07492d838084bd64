cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"
scripts/gpurun/gpu_steps.sh \
 200 "rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_c.log 2>&1" \
 200 "rocprofv3 --kernel-trace --stats -d gpurun_out/prof_in -- python3 bench.py --model imagenet_resnet50 --steps 10 --warmup 3 > gpurun_out/prof_in.log 2>&1" \
 120 "timeout -s KILL 110 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_in -- python3 bench.py --model imagenet_resnet50 --steps 2 --warmup 1 > gpurun_out/pmc_in.log 2>&1" \
 120 "timeout -s KILL 110 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_c -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/pmc_c.log 2>&1"
