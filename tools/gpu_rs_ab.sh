#!/bin/bash
# Round-4 A/B of a raw-run variant (CPK_RUN_SPLIT, measured and not kept: DESIGN.md section 4):
# GPU tests on capnproto_amd/var_rs.so, the C5 FETCH ablation on it and on the base library, and
# kernel times for both.  The variant's source change is not in the tree; var_rs.so was built
# from it with tools/build_variant.sh rs "-DCPK_RUN_SPLIT=1".
set -o pipefail
mkdir -p gpurun_out
cp capnproto_amd/libcpk_hip.so /tmp/base.so
cp capnproto_amd/var_rs.so capnproto_amd/libcpk_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_unpack.py tests/test_gpu_stream.py tests/test_gpu_configs.py -m gpu -k "not full_size and not geometric" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04z_rs_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r04z_rs_tests.log; [ $rc = 0 ] || { cp /tmp/base.so capnproto_amd/libcpk_hip.so; exit 1; }
SKIPS=0 bash tools/gpu_ablate_fetch.sh r04z_rs c5 || exit 1
cp /tmp/base.so capnproto_amd/libcpk_hip.so
SKIPS=0 bash tools/gpu_ablate_fetch.sh r04z_base c5 || exit 1
rm -rf gpurun_out/r04z_*_s0/
VARIANTS="base rs" CFGS="c5 c3 c2" bash tools/gpu_prof_ab.sh r04z; rc=$?; find gpurun_out -name "*kernel_trace.csv" -delete; exit $rc
