#!/bin/bash
# Round 3: split-K / tile-count A/B on the roofline (latency hiding through more workgroups).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for t in "" "splitk=4" "splitk_tiles=512" "splitk=4,splitk_tiles=1024" "splitk=1"; do
  DTR_TUNE="$t" timeout -k 10 200 python3 scripts/roofline.py 5 > "gpurun_out/roof_sk_${t//[=,]/_}.md" 2>&1 || exit $?
  echo "== $t"; tail -3 "gpurun_out/roof_sk_${t//[=,]/_}.md"
done
