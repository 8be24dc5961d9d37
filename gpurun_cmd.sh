cd $GRAFT_REPO_ROOT
TESTS=none CFGS="c2 c4" bash tools/gpu_check.sh f18
