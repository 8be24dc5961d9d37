"""Diagnostic: pack tiny chunks with kernel printf (CPK_DEBUG_SKIP=256)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, capnproto_amd
c = capnproto_amd.Codec(0)
for hexw in ["0103020405070608", "00000000000000000103020405070608"]:
    b = bytes.fromhex(hexw)
    w = torch.tensor(np.frombuffer(b, dtype=np.int64).copy(), device=c.device)
    off = torch.tensor([0, w.numel()], dtype=torch.int64, device=c.device)
    out, oo = c.pack_chunks(w, off)
    c.sync()
    n = int(oo[-1].item())
    print(hexw, "->", out[:n].cpu().numpy().tobytes().hex(), flush=True)
