#!/bin/bash
# timing ablations (outputs meaningless when a stage is skipped)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for sk in 0 1; do
  CPK_DEBUG_SKIP=$sk timeout -k 10 300 python - <<'PY'
import os, sys, time
sys.path.insert(0, '.')
import torch, capnproto_amd
c = capnproto_amd.Codec(0)
off, total = c.gen_offsets(4096, nseg=1, seg_words=8191, seed=1)
w = c.gen_messages('flat', off, total, nseg=1, seed=1)
cap = c.packed_bound(total, 8192) + 64
out = torch.zeros(cap + (1 << 28), dtype=torch.uint8, device=c.device)
moff = torch.empty(4097, dtype=torch.int64, device=c.device)
c.pack_messages(w, off, out=out, msg_out_off=moff); torch.cuda.synchronize()
P = 129482452
back = torch.empty(total, dtype=torch.int64, device=c.device)
c.timing(True)
for _ in range(10):
    c.pack_messages(w, off, out=out, msg_out_off=moff)
    c.unpack_messages(out, moff, total, nbytes=P, words=back)
torch.cuda.synchronize()
pm, pl, um, ul = c.timing_read()
print("skip", os.environ.get("CPK_DEBUG_SKIP"), "pack ms", pm / pl, "unpack ms", um / ul)
PY
done
