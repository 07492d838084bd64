#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 scripts/bnb_cost.py 20 > gpurun_out/bnb_cost.md 2>&1; ec=$?; cat gpurun_out/bnb_cost.md; exit $ec
