"""Times pack and unpack of the C2 batch (cpk timing events); argv[1] is a label."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, capnproto_amd
cfg = sys.argv[2] if len(sys.argv) > 2 else "c2"
c = capnproto_amd.Codec(0)
shapes = {"c2": (4096, 1, 8191, "flat"), "c3": (1 << 20, 1, 511, "flat"), "c4": (256, 16, 524288, "pointer")}
n, nseg, sw, prof = shapes[cfg]
off, total = c.gen_offsets(n, nseg=nseg, seg_words=sw, seed=1)
w = c.gen_messages(prof, off, total, nseg=nseg, seed=1)
cap = c.packed_bound(total, n * (nseg + 2)) + 64
out = torch.zeros(cap, dtype=torch.uint8, device=c.device)
moff = torch.empty(n + 1, dtype=torch.int64, device=c.device)
back = torch.empty(total, dtype=torch.int64, device=c.device)
for _ in range(3):
    c.pack_messages(w, off, out=out, msg_out_off=moff)
P = int(moff[-1].item())
for _ in range(3):
    c.unpack_messages(out, moff, total, nbytes=P, words=back)
torch.cuda.synchronize()
ok = torch.equal(back, w)
c.timing(True)
for _ in range(10):
    c.pack_messages(w, off, out=out, msg_out_off=moff)
for _ in range(10):
    c.unpack_messages(out, moff, total, nbytes=P, words=back)
torch.cuda.synchronize()
allt = c.timing_read_all()
(pm, pl), (um, ul) = allt["pack"], allt["unpack"]
U = total * 8
print(f"{sys.argv[1]} {cfg}: pack {pm / pl:.4f} ms ({U / (pm / pl) / 1e6:.0f} GB/s of U)  "
      f"unpack {um / ul:.4f} ms  P/U {P / U:.3f}  roundtrip_ok {ok}")
print("   kernels (ms): " + "  ".join(f"{k} {v[0] / v[1]:.4f}" for k, v in allt.items() if v[1]))
