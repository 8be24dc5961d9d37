#!/bin/bash
# PMC passes over one bench config: each pass is its own rocprofv3 run (counters + kernel trace
# only), then a per-kernel summary and the HBM traffic file bench.py reads (profiles/traffic_CFG).
#   gpurun --timeout 900 -- bash tools/gpu_pmc3.sh TAG CFG
set -o pipefail
TAG=${1:-pmc}
CFG=${2:-c2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_p$i" -o run \
    -- python3 "$R/bench.py" --config $CFG --sub none --steps 2 --warmup 1 --no-cpu-baseline --no-host --no-split > "$R/gpurun_out/${TAG}_p$i.log" 2>&1 \
    || { echo "pass $i failed"; tail -5 "$R/gpurun_out/${TAG}_p$i.log"; exit 1; }
  echo "pass $i done"
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out" "$TAG" "$CFG" > "$R/gpurun_out/${TAG}_summary.txt" 2>&1
cat "$R/gpurun_out/${TAG}_summary.txt"
# (the passes' raw traces stay on the box: gpurun copies back at most 64 MiB)
[ -n "$KEEP_RAW" ] || rm -rf "$R/gpurun_out/${TAG}"_p[0-9]
