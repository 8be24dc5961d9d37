#!/usr/bin/env python3
"""Diagnostic: per-kernel times of one config's pack + unpack with the CPK_DEBUG_SKIP ablation
bits of the environment (outputs are meaningless when bits are set; never a bench number).
    CPK_DEBUG_SKIP=32 python tools/ablate.py c2"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capnproto_amd  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
n, nseg, sw, prof = {"c2": (4096, 1, 8191, "flat"), "c3": (1 << 18, 1, 511, "flat"),
                     "c4": (32, 16, 524288, "pointer"), "c5": (1 << 19, 1, 0, "mixed")}[cfg]
codec = capnproto_amd.Codec(0)
off, total = codec.gen_offsets(n, nseg=nseg, seg_words=sw, seed=20261015)
words = codec.gen_messages(prof, off, total, nseg=nseg, seed=20261015)
packed, moff, st = codec.pack_messages(words, off)
codec.sync()
P = int(moff[-1].item())
codec.timing(True)
for rep in range(6):
    if rep == 2:
        codec.timing_read_all()
    codec.pack_messages(words, off, out=packed, msg_out_off=moff)
    codec.unpack_messages(packed, moff, total, nbytes=P)
    codec.sync()
tm = codec.timing_read_all()
print(cfg, "skip", os.environ.get("CPK_DEBUG_SKIP", "0"),
      {k: round(v[0] / v[1], 4) for k, v in tm.items() if v[1]})
