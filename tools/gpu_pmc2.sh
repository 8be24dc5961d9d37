#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p "$R/gpurun_out"; export TMPDIR=/tmp; cd /tmp
MODE=${1:-pack}
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU" \
           "SQ_IFETCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$R/gpurun_out/pmc2_$MODE$i" -o run -- python "$R/tools/pack_only.py" $MODE > "$R/gpurun_out/pmc2_$MODE$i.log" 2>&1 || echo "pass $i failed"
done
echo done
