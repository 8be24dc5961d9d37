#!/bin/bash
# Unpack tile kernel time by phase, without profiler: tools/ablate.py under each CPK_DEBUG_SKIP
# value in SKIPS (512 the launch alone, 64 + staging and message window, 128 + chain 0, 256 +
# entry and look-back, 0 all) for each config in CFGS.  Diagnostic only.
#   gpurun -- 'CFGS="c2 c3" bash tools/gpu_ablate_time.sh'
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for c in ${CFGS:-c2 c3}; do
  for s in ${SKIPS:-512 64 128 256 0}; do
    CPK_DEBUG_SKIP=$s timeout -k 10 120 python tools/ablate.py $c 2>&1 | grep skip || exit 1
  done
done
