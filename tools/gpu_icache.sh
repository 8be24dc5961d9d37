#!/bin/bash
# Instruction-cache counters of one bench config (one rocprofv3 pass per counter pair).
#   gpurun -- 'bash tools/gpu_icache.sh TAG CFG'
set -o pipefail
TAG=${1:-ic}
CFG=${2:-c2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVES" "SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"; do
  i=$((i+1))
  env $ENV timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_p$i" -o run \
    -- python3 "$R/bench.py" --config $CFG --sub none --steps 2 --warmup 1 --no-cpu-baseline --no-host --no-split --no-verify > "$R/gpurun_out/${TAG}_p$i.log" 2>&1 \
    || { echo "pass $i failed"; tail -5 "$R/gpurun_out/${TAG}_p$i.log"; exit 1; }
done
python3 - "$R/gpurun_out" "$TAG" <<'PY'
import csv, glob, sys
from collections import defaultdict
out, tag = sys.argv[1], sys.argv[2]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{out}/{tag}_p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r.get("Kernel_Name", "")
        k = "unpack_tiles" if "unpack_tiles_kernel<false, 0>" in n else ("pack_tile" if "pack_tile_kernel" in n else None)
        if k:
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print("==", k, {c: round(sum(v) / len(v)) for c, v in sorted(d.items())})
PY
