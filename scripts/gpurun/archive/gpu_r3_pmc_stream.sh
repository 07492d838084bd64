#!/bin/bash
# Round 3: measured HBM bytes of the streaming 1x1 kernels vs the implicit-GEMM ones (PMC).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for s in fwd1x1_probe bap_probe; do
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_$s.a -o pmc -- python3 scripts/$s.py 3 > gpurun_out/pmc_$s.a.log 2>&1 || exit 1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_$s.b -o pmc -- python3 scripts/$s.py 3 > gpurun_out/pmc_$s.b.log 2>&1 || exit 1
  a=$(find gpurun_out/pmc_$s.a -name "*counter_collection.csv" | head -1); b=$(find gpurun_out/pmc_$s.b -name "*counter_collection.csv" | head -1)
  [ -z "$a" ] && a=$(find gpurun_out/pmc_$s.a -name "*.csv" | head -1)
  [ -z "$b" ] && b=$(find gpurun_out/pmc_$s.b -name "*.csv" | head -1)
  python3 scripts/pmc_stream.py gpurun_out/pmc_$s.md "bnd1x1|bnf1x1|bn_bwd_apply|conv_gemm|conv_ring" "$a" "$b" || exit 1
  rm -rf gpurun_out/pmc_$s.a gpurun_out/pmc_$s.b
done
