#!/bin/bash
# Stream-split kernel times per library variant (VARIANTS: base = in-tree, NAME = var_NAME.so):
#   gpurun -- 'VARIANTS="base r5" bash tools/gpu_split_prof_ab.sh TAG'
set -o pipefail
TAG=${1:-spab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
cp capnproto_amd/libcpk_hip.so /tmp/cpk_base.so
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then cp /tmp/cpk_base.so capnproto_amd/libcpk_hip.so
  else cp capnproto_amd/var_$v.so capnproto_amd/libcpk_hip.so; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG}_$v" -o run \
    -- python3 "$R/tools/split_prof.py" > "$R/gpurun_out/${TAG}_$v.log" 2>&1) || { echo "prof $v failed"; tail -5 gpurun_out/${TAG}_$v.log; exit 1; }
  python3 - "$R/gpurun_out/${TAG}_$v/run_kernel_stats.csv" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if "cpk" in n and ("split" in n or "unpack" in n or "walk" in n or "meet" in n or "resolve" in n):
        print(sys.argv[2], f'{float(r["AverageNs"])/1e3:10.1f} us x{r["Calls"]:>4}  {n[:80]}')
PY
done
cp /tmp/cpk_base.so capnproto_amd/libcpk_hip.so
