#!/bin/bash
# Persistent-step variants without tune keys (forward slices, optimizer tile budget).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
timeout -k 10 300 python scripts/persist_variants.py 128 200 && timeout -k 10 300 python scripts/persist_variants.py 64 200
