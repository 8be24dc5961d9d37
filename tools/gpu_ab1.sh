set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
cp capnproto_amd/libcpk_hip.so /tmp/base.so
cp capnproto_amd/var_t.so capnproto_amd/libcpk_hip.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_t_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04_t_tests.log
cp /tmp/base.so capnproto_amd/libcpk_hip.so
[ $rc = 0 ] || exit 1
VARIANTS="base t" CFGS="c2 c4 c3" bash tools/gpu_prof_ab.sh r04ab1
SKIPS="0 4 8 16 32 48" bash tools/gpu_ablate_pmc.sh r04abp c2
