#!/bin/bash
# Kernel times (tools/ablate.py: pack and unpack_tiles per call, HIP events) of library variants
# VARIANTS (capnproto_amd/var_NAME.so; base = the in-tree build) on CFGS.  Diagnostic A/B only:
# ablation variants may produce wrong bytes, which ablate.py does not check.
#   gpurun -- 'VARIANTS="base a b" CFGS="c2 c4" bash tools/gpu_var_time.sh'
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
cp capnproto_amd/libcpk_hip.so /tmp/cpk_base.so
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then cp /tmp/cpk_base.so capnproto_amd/libcpk_hip.so
  else cp capnproto_amd/var_$v.so capnproto_amd/libcpk_hip.so; fi
  for c in ${CFGS:-c2}; do
    echo -n "$v "; timeout -k 10 120 python tools/ablate.py $c 2>&1 | grep skip || { cp /tmp/cpk_base.so capnproto_amd/libcpk_hip.so; exit 1; }
  done
done
cp /tmp/cpk_base.so capnproto_amd/libcpk_hip.so
