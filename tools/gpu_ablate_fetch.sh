#!/bin/bash
# Where the unpack tile kernel's reads beyond P come from: FETCH_SIZE (x2, the gfx950 wide-read
# correction) of unpack_tiles per CPK_DEBUG_SKIP ablation (diagnostic: outputs are wrong with
# bits set; 8 = no look-back, 64 = staging and message window only, 128 = + chain 0).
#   gpurun -- 'SKIPS="0 8 128 64" bash tools/gpu_ablate_fetch.sh TAG c3'
set -o pipefail
TAG=${1:-abf}
CFG=${2:-c3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
for s in ${SKIPS:-0}; do
  CPK_DEBUG_SKIP=$s timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
    -d "$R/gpurun_out/${TAG}_s$s" -o run -- python3 "$R/tools/ablate.py" $CFG > "$R/gpurun_out/${TAG}_s$s.log" 2>&1 \
    || { echo "skip $s failed"; tail -5 "$R/gpurun_out/${TAG}_s$s.log"; exit 1; }
  python3 - "$R/gpurun_out/${TAG}_s$s" "$s" <<'PY'
import csv, glob, sys
from collections import defaultdict
per = defaultdict(float); disp = set()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "unpack_tiles" not in r.get("Kernel_Name", ""):
            continue
        disp.add(r["Dispatch_Id"]); per[r["Counter_Name"]] += float(r["Counter_Value"] or 0)
n = max(1, len(disp))
print("skip", sys.argv[2], "unpack_tiles FETCH_SIZE x2 per launch MB", round(2 * per["FETCH_SIZE"] / n / 1e3, 1), "launches", n)
PY
done
