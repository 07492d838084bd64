# round 6: how the runtime takes ROC_GLOBAL_CU_MASK (mask words, placement per variant)
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out &&
timeout -k 10 300 python -u scripts/cu_mask_probe.py > gpurun_out/cu_mask_probe.json 2> gpurun_out/cu_mask_probe.err
EC=$?; cut -c1-4000 gpurun_out/cu_mask_probe.json; exit $EC
