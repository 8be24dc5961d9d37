#!/bin/bash
# Round-end parity evidence: every GPU test (slow ones included) and smoke, on the in-tree build.
#   gpurun --timeout 1200 -- bash tools/gpu_tests_all.sh TAG
set -o pipefail
TAG=${1:-r04}
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/${TAG}_tests_all.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_tests_all.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
