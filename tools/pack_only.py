import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, capnproto_amd
c = capnproto_amd.Codec(0)
off, total = c.gen_offsets(4096, nseg=1, seg_words=8191, seed=1)
w = c.gen_messages('flat', off, total, nseg=1, seed=1)
cap = c.packed_bound(total, 8192) + 64
out = torch.zeros(cap, dtype=torch.uint8, device=c.device)
moff = torch.empty(4097, dtype=torch.int64, device=c.device)
for _ in range(3):
    c.pack_messages(w, off, out=out, msg_out_off=moff)
P = int(moff[-1].item())
back = torch.empty(total, dtype=torch.int64, device=c.device)
if len(sys.argv) > 1 and sys.argv[1] == "unpack":
    for _ in range(3):
        c.unpack_messages(out, moff, total, nbytes=P, words=back)
torch.cuda.synchronize()
