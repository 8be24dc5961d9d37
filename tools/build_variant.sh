#!/bin/bash
# A/B builds: tools/build_variant.sh NAME "-DKNOB=V ..." compiles the library with extra defines
# into capnproto_amd/var_NAME.so (git-ignored; gpu_check.sh / gpu_prof_ab.sh VARIANTS="NAME ..."
# swap it in on the GPU box).  Fails if any source fails to compile.
set -e
NAME=$1; DEFS=$2
R=$(cd "$(dirname "$0")/.." && pwd)
B=/tmp/cpk_var_$NAME; rm -rf $B; mkdir -p $B
pids=()
for f in $R/capnproto_amd/csrc/*.hip $R/capnproto_amd/csrc/*.cpp; do
  case $f in *cpk_convert.cpp) continue;; esac
  o=$B/$(basename $f).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC $DEFS -c $f -o $o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "compile failed ($NAME)"; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/capnproto_amd/var_$NAME.so $B/*.o
echo built var_$NAME.so
