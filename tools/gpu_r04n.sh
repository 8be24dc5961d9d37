cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out; PWD_R=$(pwd)
timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04n_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04n_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python3 tools/diag_unpack.py capnproto_amd/var_diag.so split > gpurun_out/r04n_diag_split.log 2>&1 || { tail -5 gpurun_out/r04n_diag_split.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04n_diag_split.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD_R/gpurun_out/r04n_split" -o run \
    -- python3 "$PWD_R/tools/split_prof.py" > "$PWD_R/gpurun_out/r04n_split.log" 2>&1) || { echo "split prof failed"; tail -5 gpurun_out/r04n_split.log; exit 1; }
tail -3 gpurun_out/r04n_split.log
SKIPS="64 128 256 0" bash tools/gpu_ablate_pmc.sh r04n_c3 c3 && SKIPS="64 128 256 0" bash tools/gpu_ablate_pmc.sh r04n_c2 c2
