#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 > gpurun_out/ab2_tests.log 2>&1 || { tail -30 gpurun_out/ab2_tests.log; exit 1; }
tail -1 gpurun_out/ab2_tests.log
for st in 16 8; do for sk in 0 1; do
  CPK_PACK_STEPS=$st CPK_DEBUG_SKIP=$sk timeout -k 10 300 python - <<'PY'
import os, sys
sys.path.insert(0, '.')
import torch, capnproto_amd
c = capnproto_amd.Codec(0)
off, total = c.gen_offsets(4096, nseg=1, seg_words=8191, seed=1)
w = c.gen_messages('flat', off, total, nseg=1, seed=1)
cap = c.packed_bound(total, 8192) + 64
out = torch.zeros(cap + (1 << 28), dtype=torch.uint8, device=c.device)
moff = torch.empty(4097, dtype=torch.int64, device=c.device)
for _ in range(3): c.pack_messages(w, off, out=out, msg_out_off=moff)
torch.cuda.synchronize()
c.timing(True)
for _ in range(10): c.pack_messages(w, off, out=out, msg_out_off=moff)
torch.cuda.synchronize()
pm, pl, um, ul = c.timing_read()
print("steps", os.environ["CPK_PACK_STEPS"], "skip", os.environ.get("CPK_DEBUG_SKIP"), "pack ms %.4f" % (pm / pl))
PY
done; done
CPK_STAMPS=1 timeout -k 10 300 python tools/stamps.py c2 2>&1 | head -8
