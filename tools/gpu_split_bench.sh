#!/bin/bash
# The default bench line's stream split (and C2), CPU baseline and host-inclusive rate off:
#   gpurun -- 'bash tools/gpu_split_bench.sh TAG'
set -o pipefail
TAG=${1:-sb}
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --ab --sub none --steps 10 --warmup 2 --no-cpu-baseline --no-host \
  > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}.err; exit 1; }
python3 - gpurun_out/${TAG}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C2", d["value"], "split", json.dumps(d.get("stream_split"))[:400])
PY
