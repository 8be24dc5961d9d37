#!/bin/bash
# Diagnostic build counters / phase stamps (CPK_STAMPS=1) for the given configs.
#   gpurun --timeout 600 -- bash tools/gpu_diag.sh TAG "c2 c4 c5"
set -o pipefail
TAG=${1:-diag}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for c in ${2:-c2 c4}; do
  CPK_STAMPS=1 timeout -k 10 200 python tools/stamps.py $c > gpurun_out/${TAG}_$c.log 2>&1 \
    || { echo "stamps $c failed"; tail -20 gpurun_out/${TAG}_$c.log; exit 1; }
  echo "== $c"; grep -v amdgpu.ids gpurun_out/${TAG}_$c.log
done
