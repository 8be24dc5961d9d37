#!/bin/bash
# Instruction attribution of the unpack tile kernel by phase: one rocprofv3 counter pass (SQ
# instruction and cycle counters + kernel trace) of tools/ablate.py per CPK_DEBUG_SKIP value in
# SKIPS (diagnostic only: outputs are meaningless with bits set).
#   gpurun -- 'SKIPS="0 4 16 32 48" bash tools/gpu_ablate_pmc.sh TAG c2'  (PMC: another counter set)
set -o pipefail
TAG=${1:-abp}
CFG=${2:-c2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
for s in ${SKIPS:-0}; do
  CPK_DEBUG_SKIP=$s timeout -s KILL 120 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT} \
    --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_s$s" -o run \
    -- python3 "$R/tools/ablate.py" $CFG > "$R/gpurun_out/${TAG}_s$s.log" 2>&1 \
    || { echo "skip $s failed"; tail -5 "$R/gpurun_out/${TAG}_s$s.log"; exit 1; }
  tail -1 "$R/gpurun_out/${TAG}_s$s.log"
  python3 - "$R/gpurun_out/${TAG}_s$s" "$s" <<'PY'
import csv, glob, sys
from collections import defaultdict
per = defaultdict(float); disp = set()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "unpack_tiles" not in r.get("Kernel_Name", ""):
            continue
        disp.add(r["Dispatch_Id"]); per[r["Counter_Name"]] += float(r["Counter_Value"] or 0)
n = max(1, len(disp)); w = per["SQ_WAVES"] / n
print("skip", sys.argv[2], "unpack_tiles per wave:", {k: round(v / n / max(w, 1), 1) for k, v in sorted(per.items()) if k != "SQ_WAVES"}, "waves", w)
PY
done
