# round 6: the world-2 persistent overlap path on CU halves of one GPU (DTR_CU_PARTITION=2,
# shm transport): dp_check RN50 bs16/rank fp32 + bf16 exchange (20 steps), bench --gpus 2
# at global 32 / 64 / 128, the one-rank fault test, then the 1-GPU headline bench
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
export DTR_DIST_BACKEND=gloo DTR_COMM_TRANSPORT=shm DTR_CU_PARTITION=2 HSA_ENABLE_IPC_MODE_LEGACY=0 &&
for dt in fp32 bf16; do
  DP_CHECK_SIZE=50 DP_CHECK_BATCH=16 DP_CHECK_STEPS=20 DP_CHECK_ALLREDUCE=$dt timeout -k 10 300 \
    python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29801 scripts/dp_check.py > gpurun_out/r6_dp_$dt.log 2>&1 || exit 1
done &&
for gb in 32 64 128; do
  timeout -k 10 300 python -u bench.py --gpus 2 --batch $gb --steps 200 --warmup 20 > gpurun_out/r6_bench2_gb$gb.json 2> gpurun_out/r6_bench2_gb$gb.err || exit 1
done &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_dp_gpu.py -k one_rank > gpurun_out/r6_fault.log 2>&1 &&
unset DTR_DIST_BACKEND DTR_COMM_TRANSPORT DTR_CU_PARTITION &&
timeout -k 10 200 python -u bench.py > gpurun_out/r6_bench1.json 2> gpurun_out/r6_bench1.err
EC=$?; grep -h "dp_check\|DP_CHECK" gpurun_out/r6_dp_*.log; cut -c1-400 gpurun_out/r6_bench2_*.json gpurun_out/r6_bench1.json; tail -3 gpurun_out/r6_fault.log; exit $EC
