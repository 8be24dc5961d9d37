#!/bin/bash
# A/B of environment knobs on the GPU box: for each ENVS entry ("base" or "K=V,K2=V2"), short
# bench runs of the configs in CFGS (default c2 c4) printing per-kernel times.
#   gpurun -- 'ENVS="base CPK_DEBUG_SKIP=1" bash tools/gpu_env_ab.sh TAG'
set -o pipefail
TAG=${1:-ab}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
for e in ${ENVS:-base}; do
  for c in ${CFGS-c2 c4}; do
    envs=""; [ "$e" != base ] && envs=$(echo "$e" | tr ',' ' ')
    n=$(echo "$e" | tr '=,' '__')
    env $envs timeout -k 10 300 python bench.py --config $c --sub none --steps ${STEPS:-10} --warmup 2 \
      --no-cpu-baseline --ab > gpurun_out/${TAG}_${n}_$c.json 2> gpurun_out/${TAG}_${n}_$c.err \
      || { echo "bench $e $c failed"; tail -20 gpurun_out/${TAG}_${n}_$c.err; exit 1; }
    python - gpurun_out/${TAG}_${n}_$c.json "$e" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline"]["kernels"]
print(sys.argv[2], d["config"]["workload"][:3], "GiB/s", d["value"], "ms", d["ms_per_step"],
      {n: v["ms"] for n, v in k.items()})
PY
  done
done
