# schedule-perturbation race check + the GPU suites touched by the LDS-weight change
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
scripts/gpu_steps.sh \
 300 "python -u -m pytest tests/test_racecheck_gpu.py -x -v --timeout 250 --timeout-method thread > gpurun_out/t_race.log 2>&1" \
 200 "python -u -m distributed_tensorflow_resnet_amd.utils.racecheck --model cifar_resnet50 --batch 128 --steps 3 --trials 3 > gpurun_out/race_c128.log 2>&1" \
 600 "python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread --deselect tests/test_racecheck_gpu.py > gpurun_out/t_all.log 2>&1"
