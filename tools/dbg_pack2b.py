"""Diagnostic: C4-shaped messages through cpk_pack_messages vs the oracle, first mismatch."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import capnproto_amd  # noqa: E402
import pyoracle as P  # noqa: E402
from gpu_util import host_u8  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
codec = capnproto_amd.Codec(0)
o = P.Oracle()
off, total = codec.gen_offsets(n, nseg=16, seg_words=524288, seed=20261015)
words = codec.gen_messages("pointer", off, total, nseg=16, seed=20261015)
packed, moff, st = codec.pack_messages(words, off)
codec.sync()
P_ = int(moff[-1].item())
got = bytes(host_u8(packed[:P_]))
w = words[:total].cpu().numpy().view(np.uint64)
ref, roff, rst = o.pack_batch(w, off.cpu().numpy().astype(np.uint64))
ref = bytes(ref)
print("len", len(got), len(ref))
for i in range(min(len(got), len(ref))):
    if got[i] != ref[i]:
        print("first byte mismatch at", i, "got", got[i - 8:i + 8].hex(), "ref", ref[i - 8:i + 8].hex())
        break
# which word / tile: scan the oracle attribution by packing prefixes chunkwise is costly; report
# the packed position of each tile start from the debug tables instead
import ctypes as C  # noqa: E402
L = codec.lib
nt = 20000
bt = (C.c_uint64 * nt)()
tb = (C.c_uint32 * nt)()
sb = (C.c_uint8 * (16 * nt))()
L.cpk_debug_pack_tables.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
L.cpk_debug_pack_tables(codec.ctx, bt, tb, sb, nt)
cum = np.cumsum([0] + list(bt))
t = int(np.searchsorted(cum, i, side="right") - 1)
print("mismatch in tile", t, "tile starts at byte", cum[t], "tile bytes", bt[t], "tile_b", hex(tb[t]),
      "steps", list(sb[16 * t:16 * t + 16]))
