#!/bin/bash
# Parity tests, then bench lines (no CPU baseline) and diagnostic counters.
#   gpurun --timeout 900 -- bash tools/gpu_quick2.sh TAG "c2 c4" "c4b c5"
set -o pipefail
TAG=${1:-q}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
fi
for c in ${2:-c2}; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err \
    || { echo "bench $c failed"; tail -5 gpurun_out/${TAG}_bench_$c.err; exit 1; }
  python - "$c" gpurun_out/${TAG}_bench_$c.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); r=d["roofline"]
print(sys.argv[1], d["value"], "GiB/s", d["parity"], "P/U", d["config"]["packed_ratio"], {k: v["ms"] for k, v in r["kernels"].items()})
PY
done
for c in ${3:-}; do
  CPK_STAMPS=1 timeout -k 10 200 python tools/stamps.py $c > gpurun_out/${TAG}_st_$c.log 2>&1 \
    || { echo "stamps $c failed"; tail -20 gpurun_out/${TAG}_st_$c.log; exit 1; }
  echo "== $c"; grep counters gpurun_out/${TAG}_st_$c.log
done
