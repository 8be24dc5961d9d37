#!/bin/bash
# Quick A/B on the GPU box: GPU parity tests (TESTS, default all -m gpu; "none" to skip), then
# short bench runs of the configs in CFGS (default c2 c4) printing the per-kernel times, once
# per library variant in VARIANTS (default: the in-tree build; NAME = capnproto_amd/var_NAME.so
# from tools/build_variant.sh, copied over the library in this scratch copy of the repo).
#   gpurun -- 'TESTS=none VARIANTS="base a b" bash tools/gpu_check.sh TAG'
set -o pipefail
TAG=${1:-chk}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
if [ "${TESTS-all}" != "none" ]; then
  T=${TESTS:-tests}; [ "$T" = all ] && T=tests
  timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
cp capnproto_amd/libcpk_hip.so /tmp/cpk_base.so
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then cp /tmp/cpk_base.so capnproto_amd/libcpk_hip.so
  else cp capnproto_amd/var_$v.so capnproto_amd/libcpk_hip.so; fi
  for c in ${CFGS-c2 c4}; do
    timeout -k 10 300 python bench.py --config $c --sub none --steps ${STEPS:-10} --warmup 2 --no-split \
      --no-cpu-baseline > gpurun_out/${TAG}_${v}_$c.json 2> gpurun_out/${TAG}_${v}_$c.err \
      || { echo "bench $v $c failed"; tail -20 gpurun_out/${TAG}_${v}_$c.err; exit 1; }
    python - gpurun_out/${TAG}_${v}_$c.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels"]
print(sys.argv[2], d["config"]["workload"][:3], "GiB/s", d["value"], "ms", d["ms_per_step"],
      {n: v["ms"] for n, v in k.items()})
PY
  done
done
cp /tmp/cpk_base.so capnproto_amd/libcpk_hip.so
