# roctx phase markers + kernel trace of the CIFAR RN50 bench (bench --roctx)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --marker-trace --kernel-trace --stats --output-format csv -d gpurun_out/prof_mk -- python3 bench.py --roctx --steps 20 --warmup 5 > gpurun_out/prof_mk.log 2>&1
