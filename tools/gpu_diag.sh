set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for c in c2 c4 c5; do
CPK_STAMPS=1 timeout -k 10 120 python tools/stamps.py $c > gpurun_out/diag_stamps_$c.log 2>&1 || exit 1
CPK_STAMPS=1 timeout -k 10 120 python tools/stamps_idx.py ${c/c5/c3} > gpurun_out/diag_idx_$c.log 2>&1 || exit 1
done
cat gpurun_out/diag_*.log
