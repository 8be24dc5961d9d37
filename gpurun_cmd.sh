cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/f15_tests.log 2>&1; tail -2 gpurun_out/f15_tests.log; grep -E "^FAILED" gpurun_out/f15_tests.log | head -5
timeout -k 10 300 python bench.py --sub none --no-cpu-baseline > gpurun_out/f15_bench.json 2> gpurun_out/f15_bench.err; tail -c 900 gpurun_out/f15_bench.json
