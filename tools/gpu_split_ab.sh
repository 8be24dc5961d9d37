#!/bin/bash
# Stream split A/B: the bench's stream_split line (flat decode + message-chain walk) once per
# library variant in VARIANTS (base = the in-tree build; NAME = capnproto_amd/var_NAME.so).
#   gpurun -- 'VARIANTS="base mc16" bash tools/gpu_split_ab.sh TAG'
set -o pipefail
TAG=${1:-split}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cp "$R/capnproto_amd/libcpk_hip.so" /tmp/cpk_base.so
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then cp /tmp/cpk_base.so "$R/capnproto_amd/libcpk_hip.so"
  else cp "$R/capnproto_amd/var_$v.so" "$R/capnproto_amd/libcpk_hip.so"; fi
  timeout -k 10 300 python3 "$R/bench.py" --config c2 --sub none --steps 2 --warmup 1 \
    --no-cpu-baseline --no-host > "$R/gpurun_out/${TAG}_$v.log" 2>&1 \
    || { echo "bench $v failed"; tail -5 "$R/gpurun_out/${TAG}_$v.log"; cp /tmp/cpk_base.so "$R/capnproto_amd/libcpk_hip.so"; exit 1; }
  python3 - "$R/gpurun_out/${TAG}_$v.log" "$v" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln)
        s = d.get("stream_split", {})
        print("==", sys.argv[2], "split_ms", s.get("ms"), "GiBps", s.get("GiBps"), "exact", s.get("split_exact"))
PY
done
cp /tmp/cpk_base.so "$R/capnproto_amd/libcpk_hip.so"
