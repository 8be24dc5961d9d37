#!/bin/bash
# The GPU unpack / pack / config tests against a variant library (capnproto_amd/var_NAME.so).
#   gpurun -- 'bash tools/gpu_var_suite.sh NAME TAG'
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cp "$R/capnproto_amd/libcpk_hip.so" /tmp/cpk_base.so
cp "$R/capnproto_amd/var_$1.so" "$R/capnproto_amd/libcpk_hip.so"
timeout -k 10 400 python -u -m pytest "$R/tests/test_gpu_unpack.py" "$R/tests/test_gpu_pack.py" "$R/tests/test_gpu_configs.py" "$R/tests/test_gpu_stream.py" -x -q --timeout 200 --timeout-method thread > "$R/gpurun_out/$2_vsuite.log" 2>&1
rc=$?
cp /tmp/cpk_base.so "$R/capnproto_amd/libcpk_hip.so"
tail -3 "$R/gpurun_out/$2_vsuite.log"
exit $rc
