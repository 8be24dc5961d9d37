#!/bin/bash
# One gpurun call for a kernel change: the GPU tests (TESTS, default all; "none" skips) on the
# in-tree library, then a rocprof per-kernel A/B of VARIANTS on CFGS (tools/gpu_prof_ab.sh).
#   gpurun --timeout 900 -- 'VARIANTS="base old" CFGS="c2 c3" bash tools/gpu_ab.sh TAG'
set -o pipefail
TAG=${1:-ab}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
if [ "${TESTS-all}" != "none" ]; then
  T=${TESTS:-tests}; [ "$T" = all ] && T=tests
  timeout -k 10 500 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  tail -3 gpurun_out/${TAG}_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/${TAG}_tests.log | head -5
  # a failing test is information; a fault, abort or time limit ends the call
  [ $rc = 0 ] || [ $rc = 1 ] || { echo "tests rc=$rc: stopping"; exit 1; }
fi
[ -n "$VARIANTS" ] || exit 0
VARIANTS="$VARIANTS" CFGS="${CFGS:-c2 c3}" bash tools/gpu_prof_ab.sh ${TAG}
