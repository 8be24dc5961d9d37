cd $GRAFT_REPO_ROOT
for c in c2 c3 c4; do bash tools/gpu_pmc3.sh r03_$c $c > gpurun_out/r03_pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/r03_pmc_$c.log; exit 1; }; done
echo pmc done
CFGS="c2 c3 c4" bash tools/gpu_prof.sh r03p
