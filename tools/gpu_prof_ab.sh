#!/bin/bash
# Per-kernel A/B: rocprofv3 kernel-trace stats of short bench runs, once per library variant in
# VARIANTS (base = the in-tree build; NAME = capnproto_amd/var_NAME.so) and config in CFGS.
#   gpurun -- 'VARIANTS="p0 base" CFGS="c4" bash tools/gpu_prof_ab.sh TAG'
set -o pipefail
TAG=${1:-pab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cp "$R/capnproto_amd/libcpk_hip.so" /tmp/cpk_base.so
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then cp /tmp/cpk_base.so "$R/capnproto_amd/libcpk_hip.so"
  else cp "$R/capnproto_amd/var_$v.so" "$R/capnproto_amd/libcpk_hip.so"; fi
  for c in ${CFGS:-c4}; do
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_${v}_${c}" -o run \
      -- python3 "$R/bench.py" --config $c --sub none --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-host --no-split \
      > "$R/gpurun_out/${TAG}_${v}_${c}.log" 2>&1) || { echo "rocprof $v $c failed"; tail -20 "$R/gpurun_out/${TAG}_${v}_${c}.log"; exit 1; }
    grep -q "check failed\|differ from the reference" "$R/gpurun_out/${TAG}_${v}_${c}.log" && echo "!! $v $c: WRONG OUTPUT"
    f=$(find "$R/gpurun_out/${TAG}_${v}_${c}" -name '*kernel_stats.csv' | head -1)
    python3 - "$f" "$v $c" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print("==", sys.argv[2], " ".join(f'{r["Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1][:22]}={float(r["AverageNs"])/1e3:.1f}'
      for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:9] if "cpk" in r["Name"] and "copy_kernel" not in r["Name"] and "gen_" not in r["Name"]))
PY
  done
done
cp /tmp/cpk_base.so "$R/capnproto_amd/libcpk_hip.so"
