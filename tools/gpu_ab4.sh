#!/bin/bash
# tests + default bench + per-kernel A/B of VARIANTS on CFGS + unpack phase attribution (PMC)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
TAG=${1:-r04d}
bash tools/gpu_ab3.sh $TAG || exit 1
SKIPS="${SKIPS:-0 64 128 256}" bash tools/gpu_ablate_pmc.sh ${TAG}_abp c2
