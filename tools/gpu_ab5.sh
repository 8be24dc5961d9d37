#!/bin/bash
# tests + default bench + per-kernel A/B of VARIANTS on CFGS + unpack step counters (var_diag.so)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
TAG=${1:-r04f}
bash tools/gpu_ab3.sh $TAG || exit 1
if [ -f capnproto_amd/var_diag.so ]; then
  timeout -k 10 300 python3 tools/diag_unpack.py capnproto_amd/var_diag.so ${DIAG_CFGS:-c2 c3 c4} > gpurun_out/${TAG}_diag.log 2>&1
  rc=$?; cat gpurun_out/${TAG}_diag.log | tail -5; [ $rc = 0 ] || exit 1
fi
