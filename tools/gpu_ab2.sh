#!/bin/bash
# Round-4 A/B: GPU tests on the in-tree library, GPU tests with the direct-pack variant
# (capnproto_amd/var_direct.so), per-kernel rocprof A/B of the variants, PMC instruction
# attribution of the unpack tile kernel by ablation.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
TAG=${1:-r04b}
timeout -k 10 500 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_base_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_base_tests.log
[ $rc = 0 ] || [ $rc = 1 ] || exit 1   # 1 = a test failed (read the log); other codes: stop
V="base"
for v in ${CANDS:-direct}; do
  cp capnproto_amd/libcpk_hip.so /tmp/base.so
  cp capnproto_amd/var_$v.so capnproto_amd/libcpk_hip.so
  timeout -k 10 400 python -u -m pytest tests/test_gpu_pack.py tests/test_gpu_configs.py tests/test_gpu_binding.py tests/test_gpu_facade.py -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_${v}_tests.log 2>&1
  vrc=$?; tail -3 gpurun_out/${TAG}_${v}_tests.log
  cp /tmp/base.so capnproto_amd/libcpk_hip.so
  [ $vrc = 0 ] && V="$V $v"
  [ $vrc = 0 ] || [ $vrc = 1 ] || exit 1
done
VARIANTS="$V" CFGS="c2 c4 c3" bash tools/gpu_prof_ab.sh ${TAG}_ab || exit 1
SKIPS="0 4 8 16 32 48" bash tools/gpu_ablate_pmc.sh ${TAG}_abp c2
