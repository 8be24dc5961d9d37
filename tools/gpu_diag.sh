#!/bin/bash
# Per-phase stamps (CPK_STAMPS=1 builds the stamp paths in): pack3 and index kernels, plus the
# unpack event counters, for the configs in CFGS (default c2 c4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
for c in ${CFGS:-c2 c4}; do
  CPK_STAMPS=1 timeout -k 10 120 python tools/stamps_pack3.py $c > gpurun_out/diag_pack3_$c.log 2>&1 || exit 1
  CPK_STAMPS=1 timeout -k 10 120 python tools/stamps.py $c > gpurun_out/diag_stamps_$c.log 2>&1 || exit 1
  CPK_STAMPS=1 timeout -k 10 120 python tools/stamps_idx.py $c > gpurun_out/diag_idx_$c.log 2>&1 || exit 1
  cat gpurun_out/diag_pack3_$c.log gpurun_out/diag_idx_$c.log | grep -v amdgpu.ids
done
