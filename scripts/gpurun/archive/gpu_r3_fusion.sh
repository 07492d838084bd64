#!/bin/bash
# Round 3: where the fused forward / dgrad convs spend time (per fusion), after the ring.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 scripts/fwd_fusion_cost.py > gpurun_out/fwd_fusion.md 2>&1 || { tail -20 gpurun_out/fwd_fusion.md; exit 1; }
cat gpurun_out/fwd_fusion.md
timeout -k 10 300 python3 scripts/dgrad_fusion_cost.py > gpurun_out/dgrad_fusion.md 2>&1 || { tail -20 gpurun_out/dgrad_fusion.md; exit 1; }
cat gpurun_out/dgrad_fusion.md
timeout -k 10 300 python3 scripts/bn_bwd_grid.py 256 512 1024 2048 > gpurun_out/bn_bwd_grid.md 2>&1 || { tail -20 gpurun_out/bn_bwd_grid.md; exit 1; }
cat gpurun_out/bn_bwd_grid.md
