#!/bin/bash
# Quick GPU iteration: parity tests, then bench lines for the given configs (no CPU baseline).
#   gpurun --timeout 900 -- bash tools/gpu_quick.sh TAG "c2 c3"
set -o pipefail
TAG=${1:-q}
CFGS=${2:-c2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then echo "tests failed rc=$rc"; exit $rc; fi
for c in $CFGS; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/${TAG}_bench_$c.err; exit 1; }
  python - "$c" gpurun_out/${TAG}_bench_$c.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); r=d["roofline"]
print(sys.argv[1], d["value"], "GiB/s", "pack_ms", r["pack_ms"], "unpack_ms", r["unpack_ms"], "frac", r["frac"], "rt_frac", r["roundtrip_frac"], "P/U", d["config"]["packed_ratio"], d["parity"])
PY
done
