cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/f19_tests.log 2>&1; tail -2 gpurun_out/f19_tests.log; grep -E "^FAILED" gpurun_out/f19_tests.log | head -5
TESTS=none CFGS="c2 c3 c5" bash tools/gpu_check.sh f19
