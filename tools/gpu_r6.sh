#!/bin/bash
# Round-6 working check on the GPU box: GPU tests (TESTS: pytest paths, "none" to skip), bench of
# the configs in CFGS for each env setting in ENVS ("-" = defaults; e.g. "CPK_UNPACK_SPLIT=0"),
# then a rocprofv3 kernel summary of each config in PROF (default c2).
#   gpurun --timeout 900 -- 'bash tools/gpu_r6.sh TAG'
set -o pipefail
TAG=${1:-r6}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS-tests}" != "none" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 150 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
for e in ${ENVS:--}; do
  for c in ${CFGS-c2 c3 c4 c5}; do
    if [ "$e" = "-" ]; then EV=""; else EV="$e"; fi
    env $EV timeout -k 10 300 python bench.py --config $c --sub none --steps ${STEPS:-10} --warmup 2 \
      --no-split --no-host --no-cpu-baseline ${AB:+--ab} > gpurun_out/${TAG}_${c}_${e//=/_}.json \
      2> gpurun_out/${TAG}_${c}_${e//=/_}.err || { echo "bench $c $e failed"; tail -20 gpurun_out/${TAG}_${c}_${e//=/_}.err; exit 1; }
    python - gpurun_out/${TAG}_${c}_${e//=/_}.json "$e" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], d["config"]["workload"][:3], "GiB/s", d["value"], "ms", d["ms_per_step"],
      "pack", r["pack_ms"], "unpack", r["unpack_ms"])
PY
  done
done
cd /tmp
for c in ${PROF-c2}; do
  [ "$c" = none ] && continue
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_prof_$c" -o run \
    -- python3 "$R/bench.py" --config $c --sub none --steps 10 --warmup 2 --no-cpu-baseline --no-host --no-split \
    > "$R/gpurun_out/${TAG}_prof_$c.log" 2>&1 || { echo "rocprof $c failed"; tail -20 "$R/gpurun_out/${TAG}_prof_$c.log"; exit 1; }
  f="$R/gpurun_out/${TAG}_prof_$c/run_kernel_stats.csv"
  [ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"]
    if "cpk" in n and "copy_kernel" not in n:
        print(f'{float(r["AverageNs"])/1e3:10.1f} us x{r["Calls"]:>4}  {n[:90]}')
PY
done
