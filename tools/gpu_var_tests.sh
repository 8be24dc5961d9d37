#!/bin/bash
# run the stream GPU tests with a variant library swapped in
R=${GRAFT_REPO_ROOT:-$(pwd)}
cp "$R/capnproto_amd/libcpk_hip.so" /tmp/cpk_base.so
cp "$R/capnproto_amd/var_$1.so" "$R/capnproto_amd/libcpk_hip.so"
timeout -k 10 300 python -u -m pytest "$R/tests/test_gpu_stream.py" "$R/tests/test_gpu_facade.py" "$R/tests/test_gpu_convert.py" -x -q --timeout 200 --timeout-method thread > "$R/gpurun_out/$2_vtests.log" 2>&1
rc=$?
cp /tmp/cpk_base.so "$R/capnproto_amd/libcpk_hip.so"
tail -3 "$R/gpurun_out/$2_vtests.log"
exit $rc
