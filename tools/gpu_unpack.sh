#!/bin/bash
# Unpack A/B: GPU unpack + config tests, then bench lines (C2, C3, C4).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-u2}
timeout -k 10 300 python -u -m pytest tests/test_gpu_unpack.py tests/test_gpu_configs.py tests/test_gpu_facade.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for v in ${1:-BASE=1}; do
  env $(echo $v | tr ',' ' ') timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --sub c3,c4 --sub-steps 4 > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/${TAG}_$v.err; exit 1; }
  python - "$v" gpurun_out/${TAG}_$v.json <<'PY'
import json, sys
r = json.load(open(sys.argv[2]))
def line(x):
    k = x["roofline"]["kernels"]
    return f'{x["config"]["workload"][:3]} {x["value"]:8.1f} GiB/s frac {x["roofline"]["frac"]:.3f} pack {k.get("pack",{}).get("ms")} idx {k["unpack_index"]["ms"]} res {k["unpack_resolve"]["ms"]} exp {k["unpack_expand"]["ms"]}'
print(sys.argv[1]); print(" ", line(r))
for s in r.get("sub_results", []): print(" ", line(s))
PY
done
