#!/bin/bash
# Diagnostic A/B of one test under CPK_DEBUG_SKIP values.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T="tests/test_gpu_unpack.py -k round_trip_batches"
for v in 0 64 128 192; do
CPK_DEBUG_SKIP=$v timeout -k 10 120 python -u -m pytest $T -x -q --timeout 60 --timeout-method thread > gpurun_out/ab_$v.log 2>&1; echo "$v rc=$?"; tail -1 gpurun_out/ab_$v.log
done
