#!/bin/bash
# Parity tests once, then pack timing of C2 under tuning knobs (env A/B).
#   gpurun -- bash tools/gpu_ab3.sh "CPK_PACK_STEPS=8 CPK_PACK_STEPS=4,CPK_PACK_PF=1"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
VARIANTS=${1:-"CPK_PACK_STEPS=8"}
timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 > gpurun_out/ab3_tests.log 2>&1 || { tail -30 gpurun_out/ab3_tests.log; exit 1; }
tail -1 gpurun_out/ab3_tests.log
for v in $VARIANTS; do
  env $(echo $v | tr ',' ' ') timeout -k 10 300 python tools/time_c2.py "$v" || exit 1
done
