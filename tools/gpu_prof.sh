#!/bin/bash
# rocprofv3 kernel-trace stats of short bench runs, one per config in CFGS (default c2 c4):
# gpurun_out/<TAG>_<cfg>_prof/.../*kernel_stats.csv
set -o pipefail
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
for c in ${CFGS:-c2 c4}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_${c}_prof" -o run \
    -- python3 "$R/bench.py" --config $c --sub none --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-host --no-split \
    > "$R/gpurun_out/${TAG}_${c}_prof.log" 2>&1 || { echo "rocprof $c failed"; tail -20 "$R/gpurun_out/${TAG}_${c}_prof.log"; exit 1; }
  f=$(find "$R/gpurun_out/${TAG}_${c}_prof" -name '*kernel_stats.csv' | head -1)
  echo "== $c"; python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:9.2f}')
PY
done
