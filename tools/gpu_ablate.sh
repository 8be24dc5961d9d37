#!/bin/bash
# Pack/unpack ablations on the GPU box: tools/ablate.py per config in CFGS for each CPK_DEBUG_SKIP
# value in SKIPS (diagnostic only; outputs are meaningless with bits set).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for c in ${CFGS:-c2 c4}; do
  for s in ${SKIPS:-0}; do
    CPK_DEBUG_SKIP=$s timeout -k 10 120 python tools/ablate.py $c 2>&1 | tail -1 | tee -a gpurun_out/${1:-abl}.txt \
      || { echo "ablate $c $s failed"; exit 1; }
  done
done
