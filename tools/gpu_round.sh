#!/bin/bash
# One gpurun call covering the round-end evidence: parity tests, smoke, the default bench line
# (C2, with CPU baseline, host-inclusive rate, small-message latency and the stream split), bench
# lines for C3-C5, and a rocprofv3 kernel-trace summary of the default bench.
#   gpurun --timeout 1100 -- bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
fi
timeout -k 10 300 python bench.py --host-inclusive > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err \
  || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench_c2.err; exit 1; }
cat gpurun_out/${TAG}_bench_c2.json; tail -2 gpurun_out/${TAG}_bench_c2.err
for c in ${CFGS-c3 c4 c5}; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-split --no-host \
    > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err \
    || { echo "bench $c failed"; tail -20 gpurun_out/${TAG}_bench_$c.err; exit 1; }
  cat gpurun_out/${TAG}_bench_$c.json
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_prof" -o run \
  -- python3 "$R/bench.py" --sub none --steps 20 --warmup 3 --no-cpu-baseline --no-host --no-split > "$R/gpurun_out/${TAG}_prof.log" 2>&1 \
  || { echo "rocprof failed"; tail -20 "$R/gpurun_out/${TAG}_prof.log"; exit 1; }
echo "rocprof done"
# the HBM-honest configs' kernel summaries too (C3, C4)
for c in ${PROF_CFGS-c3 c4}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_prof_$c" -o run \
    -- python3 "$R/bench.py" --config $c --sub none --steps 5 --warmup 2 --no-cpu-baseline --no-host --no-split > "$R/gpurun_out/${TAG}_prof_$c.log" 2>&1 \
    || { echo "rocprof $c failed"; tail -20 "$R/gpurun_out/${TAG}_prof_$c.log"; exit 1; }
  echo "rocprof $c done"
done
