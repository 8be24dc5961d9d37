#!/bin/bash
# Pack parity tests under the A/B knobs: the step-major kernels of cpk_pack.hip (CPK_PACK3=0;
# tile steps, two-pass form), the two-pass kernel of cpk_pack2.hip (CPK_PACK_V2=1), and the
# lane-serial default with a capped grid (CPK_PACK3_BLOCKS).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for v in ${1:-CPK_PACK3=0 CPK_PACK3=0,CPK_PACK_STEPS=8 CPK_PACK3=0,CPK_PACK_TWO_PASS=1 CPK_PACK_V2=1 CPK_PACK3_BLOCKS=64}; do
  env $(echo $v | tr ',' ' ') timeout -k 10 200 python -u -m pytest tests/test_gpu_pack.py -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/knob.log 2>&1 \
    || { echo "$v failed"; tail -20 gpurun_out/knob.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/knob.log)"
done
