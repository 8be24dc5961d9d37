#!/bin/bash
# Pack/unpack timing of one config under tuning knobs (env A/B), no tests.
#   gpurun -- bash tools/gpu_ab4.sh c2 "CPK_PACK_STEPS=8 CPK_PACK_STEPS=16,CPK_PACK_PF=1"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
CFG=${1:-c2}
for v in ${2:-CPK_PACK_STEPS=8}; do
  env $(echo $v | tr ',' ' ') timeout -k 10 300 python tools/time_c2.py "$v" $CFG || exit 1
done
