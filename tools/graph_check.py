#!/usr/bin/env python3
"""Diagnostic: pack / unpack captured into a HIP graph and replayed vs eager launches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import capnproto_amd  # noqa: E402

codec = capnproto_amd.Codec(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
off, total = codec.gen_offsets(n, 1, 8191, seed=7)
words = codec.gen_messages("flat", off, total, 1, seed=7)
cap = codec.packed_bound(total, 2 * n) + 64
codec.reserve(total, cap, n)
ref, roff, _ = codec.pack_messages(words, off)
codec.sync()
P = int(roff[-1].item())
ref = ref[:P].clone()
roff = roff.clone()
packed = torch.zeros(cap, dtype=torch.uint8, device=codec.device)
moff = torch.zeros(n + 1, dtype=torch.int64, device=codec.device)
pst = torch.zeros(n, dtype=torch.int32, device=codec.device)
codec.pack_messages(words, off, out=packed, msg_out_off=moff, status=pst)
codec.sync()
print("eager pack ok:", torch.equal(packed[:P], ref), torch.equal(moff, roff))
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    codec.pack_messages(words, off, out=packed, msg_out_off=moff, status=pst)
packed.zero_()
moff.zero_()
torch.cuda.synchronize()
for r in range(3):
    g.replay()
    torch.cuda.synchronize()
    codec.sync()
    good = torch.equal(packed[:P], ref)
    print(f"graph pack replay {r}: bytes {good} offsets {torch.equal(moff, roff)}")
    if not good:
        d = (packed[:P] != ref).nonzero()
        print("  first diff at", int(d[0].item()), "count", d.numel())
back = torch.zeros(total, dtype=torch.int64, device=codec.device)
woff = torch.zeros(n + 1, dtype=torch.int64, device=codec.device)
ust = torch.zeros(n, dtype=torch.int32, device=codec.device)
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2):
    codec.unpack_messages(ref, roff, total, nbytes=P, words=back, msg_word_off=woff, status=ust)
for r in range(3):
    back.zero_()
    g2.replay()
    torch.cuda.synchronize()
    codec.sync()
    print(f"graph unpack replay {r}: words {torch.equal(back, words[:total])} status {bool((ust == 0).all())}")
# pack + unpack in one graph (the bench's step)
g3 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g3):
    codec.pack_messages(words, off, out=packed, msg_out_off=moff, status=pst)
    codec.unpack_messages(packed, moff, total, nbytes=P, words=back, msg_word_off=woff, status=ust)
for r in range(3):
    packed.zero_()
    back.zero_()
    g3.replay()
    torch.cuda.synchronize()
    codec.sync()
    print(f"graph pack+unpack replay {r}: bytes {torch.equal(packed[:P], ref)} "
          f"words {torch.equal(back, words[:total])} status {bool((ust == 0).all())}")
