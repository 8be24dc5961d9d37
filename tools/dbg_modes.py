#!/usr/bin/env python3
"""Diagnostic: the unpack modes (messages, one flat chunk, size only, stream split) on a random
batch against the oracle, printing the first mismatching word and its packed tile."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import capnproto_amd  # noqa: E402
import cases  # noqa: E402
from oracle import pyoracle as PO  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 44
nm = int(sys.argv[2]) if len(sys.argv) > 2 else 300
rng = np.random.default_rng(seed)
words, off = cases.message_batch(rng, nm, max_seg=6, max_words=900)
orc = PO.Oracle()
packed, poff, status = orc.pack_batch(words, off)
N = len(words)
Pb = len(packed)
print("words", N, "packed", Pb, "tiles", (Pb + 4095) // 4096)
c = capnproto_amd.Codec(0)
dev = c.device
dp = torch.from_numpy(np.frombuffer(packed.tobytes(), np.uint8).copy()).to(dev)
dpo = torch.from_numpy(poff.astype(np.int64)).to(dev)


def first_diff(got, want, what):
    got = np.asarray(got, dtype=np.uint64)
    want = np.asarray(want, dtype=np.uint64)
    n = min(len(got), len(want))
    bad = np.nonzero(got[:n] != want[:n])[0]
    if len(bad) == 0 and len(got) >= len(want):
        print(what, "OK")
        return
    i = int(bad[0]) if len(bad) else n
    m = int(np.searchsorted(off, i, side="right") - 1)
    print(what, "first diff at word", i, "of", len(want), "message", m, "nbad", len(bad))


w, mwo, st = c.unpack_messages(dp, dpo, N)
c.sync()
print("mode0 status nonzero:", int((st.cpu().numpy() != 0).sum()))
first_diff(w[:N].cpu().numpy().view(np.uint64), words, "mode0")
io = torch.tensor([0, Pb], dtype=torch.int64, device=dev)
sz, sst = c.unpacked_size(dp, io)
c.sync()
print("mode2 size", int(sz[0].item()), "want", N, "status", int(sst[0].item()))
wo = torch.tensor([0, N], dtype=torch.int64, device=dev)
w1, st1 = c.unpack_chunks(dp, io, wo)
c.sync()
print("mode1 status", int(st1[0].item()))
first_diff(w1[:N].cpu().numpy().view(np.uint64), words, "mode1")
ws, woff, ioff, sts, n = c.split_packed_stream(dp, N, nm + 4)
c.sync()
print("split n", int(n.item()), "status", sts[: int(n.item()) + 1].cpu().numpy()[-3:])
first_diff(ws[:N].cpu().numpy().view(np.uint64), words, "split")
if os.environ.get("CPK_STAMPS"):
    import ctypes as C
    L = c.lib
    L.cpk_debug_dump.argtypes = [C.c_int, C.POINTER(C.c_uint64), C.c_uint64]
    buf = (C.c_uint64 * 4096)()
    # one more mode-0 decode so the dump is of it
    c.unpack_messages(dp, dpo, N)
    c.sync()
    L.cpk_debug_dump(1, buf, 4096)
    for t in [int(x) for x in os.environ.get("TILES", "124,125,126,127").split(",")]:
        v = buf[4 * t: 4 * t + 4]
        print("tile", t, "E", v[0] & 0xffffffff, "Eopt", v[0] >> 32, "xE", v[1] & 0xffffffff,
              "x0", v[1] >> 32, "excl", v[2], "w", v[3] & 0xffffffff, "fms", (v[3] >> 32) & 0x7fffffff,
              "start", v[3] >> 63)
