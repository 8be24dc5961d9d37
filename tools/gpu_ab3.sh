#!/bin/bash
# GPU tests on the in-tree library, the default bench line, then a per-kernel rocprof A/B of the
# variant libraries in VARIANTS (capnproto_amd/var_NAME.so) on CFGS.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
TAG=${1:-r04c}
timeout -k 10 500 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log
[ $rc = 0 ] || [ $rc = 1 ] || exit 1
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1])
print('C2', d['value'], d['ms_per_step'], 'copy', d['roofline'].get('measured_copy_GBps'), d['roofline'].get('measured_copy_sweep_GBps'))
print('small', d.get('small_message_latency'))
print('split', d.get('stream_split',{}).get('GiBps'), 'host', d.get('host_inclusive',{}).get('pipelined',{}).get('GiBps'))
for s in d.get('sub_results',[]): print(s['config']['workload'][:3], s['value'], s['ms_per_step'], s['roofline']['pack_ms'], s['roofline']['unpack_ms'])
"
VARIANTS="${VARIANTS:-base}" CFGS="${CFGS:-c2 c3}" bash tools/gpu_prof_ab.sh ${TAG}_ab
