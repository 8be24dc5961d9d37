#!/bin/bash
# Round-end evidence in one call, on the in-tree library and sources as committed: the PMC
# traffic passes (C2, C4, C3) copied into profiles/ (stamped with the kernel source hash bench.py
# checks), then parity tests, smoke, bench lines and the rocprof summary (gpu_round.sh).
#   gpurun --timeout 1180 -- bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-r04}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for c in ${PMC_CFGS:-c2 c4 c3}; do
  bash tools/gpu_pmc3.sh ${TAG}_$c $c > gpurun_out/${TAG}_pmc_$c.out 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/${TAG}_pmc_$c.out; exit 1; }
  cp gpurun_out/${TAG}_${c}_traffic_$c.json profiles/traffic_$c.json
done
echo "pmc done"
[ -n "$PMC_ONLY" ] && exit 0
bash tools/gpu_round.sh $TAG
