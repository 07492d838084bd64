#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python3 scripts/bap_probe.py 20 > gpurun_out/bap_probe.md 2>&1; ec=$?; cat gpurun_out/bap_probe.md; exit $ec
