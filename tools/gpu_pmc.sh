#!/bin/bash
# PMC passes (each pass its own rocprofv3 run, counters only with --kernel-trace).
#   gpurun --timeout 1100 -- bash tools/gpu_pmc.sh TAG CFG
set -o pipefail
TAG=${1:-pmc}
CFG=${2:-c2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/${TAG}_counters.txt" 2>&1 || true
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_p$i" -o run -- python "$R/bench.py" --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/${TAG}_p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/${TAG}_p$i.log"; }
done
echo pmc done
