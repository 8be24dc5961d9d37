"""Diagnostic: the edge-chunk batch through cpk_pack_chunks vs the oracle, first mismatch."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import capnproto_amd  # noqa: E402
import cases  # noqa: E402
import pyoracle as P  # noqa: E402
from gpu_util import dev, host_u8  # noqa: E402

codec = capnproto_amd.Codec(0)
o = P.Oracle()
ch = cases.edge_chunks()
words = np.concatenate(ch)
off = np.cumsum([0] + [len(c) for c in ch]).astype(np.int64)
ref = b"".join(o.pack_chunk(c) for c in ch)
out, coff = codec.pack_chunks(dev(codec, words), dev(codec, off))
codec.sync()
coff = coff.cpu().numpy()
got = bytes(host_u8(out[: int(coff[-1])]))
print("len got", len(got), "ref", len(ref))
refoff = np.cumsum([0] + [len(o.pack_chunk(c)) for c in ch])
for i in range(len(ch)):
    if coff[i] != refoff[i]:
        print("first offset mismatch at chunk", i, coff[i], refoff[i])
        break
for i in range(min(len(got), len(ref))):
    if got[i] != ref[i]:
        print("first byte mismatch at", i, "got", got[i - 4:i + 8].hex(), "ref", ref[i - 4:i + 8].hex())
        break
import ctypes as C  # noqa: E402
L = codec.lib
nt = 4
bt = (C.c_uint64 * nt)()
tb = (C.c_uint32 * nt)()
sb = (C.c_uint8 * (16 * nt))()
L.cpk_debug_pack_tables.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]
print("debug rc", L.cpk_debug_pack_tables(codec.ctx, bt, tb, sb, nt))
print("tile bytes", list(bt), "tile_b", [hex(x) for x in tb])
print("step_b", list(sb))
