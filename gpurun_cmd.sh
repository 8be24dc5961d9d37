cd $GRAFT_REPO_ROOT
SKIPS="0 4 8 16 48 60" CFGS="c2 c4" bash tools/gpu_ablate.sh ab1 && TESTS=none VARIANTS="base w7" CFGS="c2 c3 c5" bash tools/gpu_check.sh f6 && CFGS="c2 c4" bash tools/gpu_prof.sh p6 && timeout -k 10 200 python -u -m pytest tests/test_gpu_pack.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k concurrent
