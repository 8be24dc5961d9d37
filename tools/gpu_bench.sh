#!/bin/bash
# One gpurun call: smoke, default bench line, rocprofv3 kernel-trace summary of the same bench.
#   gpurun --timeout 1100 -- bash tools/gpu_bench.sh [tag] [config]
set -e -o pipefail
TAG=${1:-r01}
CFG=${2:-c2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
echo "smoke done"
timeout -k 10 600 python bench.py --config $CFG --steps 20 --warmup 3 > gpurun_out/bench_${TAG}_$CFG.json 2> gpurun_out/bench_${TAG}_$CFG.err
echo "bench done"; cat gpurun_out/bench_${TAG}_$CFG.json
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}_$CFG" -o run -- python "$R/bench.py" --config $CFG --steps 10 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof_${TAG}_$CFG.log" 2>&1
echo "rocprof done"
