#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 300 ./capnproto_amd/cpk_facade_test tests/golden > gpurun_out/facade.log 2>&1; rc=$?
tail -40 gpurun_out/facade.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_pack.py tests/test_gpu_unpack.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fu_tests.log 2>&1 || { tail -30 gpurun_out/fu_tests.log; exit 1; }
tail -1 gpurun_out/fu_tests.log
