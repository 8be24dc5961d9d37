#!/bin/bash
# C4 shape with geometric zero stretches: GPU parity test against the oracle, the bench line and
# a kernel-trace summary.   gpurun --timeout 900 -- bash tools/gpu_c4g.sh TAG
set -o pipefail
TAG=${1:-r04c4g}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k geometric -x -v --timeout 240 \
  --timeout-method thread > gpurun_out/${TAG}_test.log 2>&1 || { echo "test failed"; tail -30 gpurun_out/${TAG}_test.log; exit 1; }
tail -1 gpurun_out/${TAG}_test.log
for c in c4g c4; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --sub none --no-cpu-baseline --no-split --no-host \
    > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err \
    || { echo "bench $c failed"; tail -20 gpurun_out/${TAG}_bench_$c.err; exit 1; }
  cat gpurun_out/${TAG}_bench_$c.json
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_prof" -o run \
  -- python3 "$R/bench.py" --config c4g --sub none --steps 5 --warmup 2 --no-cpu-baseline --no-host --no-split > "$R/gpurun_out/${TAG}_prof.log" 2>&1 \
  || { echo "rocprof failed"; tail -20 "$R/gpurun_out/${TAG}_prof.log"; exit 1; }
echo "rocprof done"
