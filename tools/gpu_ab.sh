#!/bin/bash
# A/B of tuning knobs on one box: bench c2 with each env setting, plus PMC for the default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for st in 16 8 4; do
  CPK_PACK_STEPS=$st timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$st.json 2>/dev/null && python -c "import json;d=json.loads(open('gpurun_out/ab_$st.json').read().strip().splitlines()[-1]);r=d['roofline'];print('steps=$st',d['value'],r['pack_ms'],r['unpack_ms'])"
done
export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d "$R/gpurun_out/ab_pmc" -o run -- python "$R/bench.py" --config c2 --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/ab_pmc.log" 2>&1 || echo pmc failed
echo done
