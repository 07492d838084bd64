# A/B: eager two-stream plan vs hipGraph (single stream / with the wgrad side stream)
set -o pipefail
for B in 128 16; do
  timeout -k 10 120 python3 bench.py --batch $B > gpurun_out/ab_eager_$B.log 2>&1 || exit $?
  timeout -k 10 120 python3 bench.py --batch $B --graph > gpurun_out/ab_graph_$B.log 2>&1 || exit $?
  DTR_FORK_WGRAD=1 timeout -k 10 120 python3 bench.py --batch $B --graph > gpurun_out/ab_graphfork_$B.log 2>&1 || exit $?
done
grep -H '"value"' gpurun_out/ab_*.log | sed 's/"data".*//'
