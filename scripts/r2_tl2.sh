cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export HSA_KERNARG_POOL_SIZE=67108864
scripts/gpu_steps.sh \
 200 "rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlk16 -- python3 bench.py --batch 16 --steps 20 --warmup 5 --phase-steps 0 > gpurun_out/tlk16.log 2>&1"
