cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out; PWD_R=$(pwd); TAG=${1:-r04o}
timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${TAG}_tests.log; [ $rc = 0 ] || exit 1
for v in base ${VARIANTS}; do
  if [ $v != base ]; then cp capnproto_amd/libcpk_hip.so /tmp/cpk_main.so; cp capnproto_amd/var_$v.so capnproto_amd/libcpk_hip.so; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD_R/gpurun_out/${TAG}_split_$v" -o run \
      -- python3 "$PWD_R/tools/split_prof.py" > "$PWD_R/gpurun_out/${TAG}_split_$v.log" 2>&1); rc=$?
  if [ $v != base ]; then cp /tmp/cpk_main.so capnproto_amd/libcpk_hip.so; fi
  [ $rc = 0 ] || { echo "split prof $v failed"; tail -5 gpurun_out/${TAG}_split_$v.log; exit 1; }
  echo "== $v"; grep "split ms" gpurun_out/${TAG}_split_$v.log
done
timeout -k 10 150 python3 tools/diag_unpack.py capnproto_amd/var_diag.so split > gpurun_out/${TAG}_diag_split.log 2>&1 || { tail -5 gpurun_out/${TAG}_diag_split.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_diag_split.log
