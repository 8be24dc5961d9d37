#!/usr/bin/env python3
"""Diagnostic: per-phase cycles of the lane-serial pack kernel (CPK_STAMPS=1)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capnproto_amd  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
n, nseg, sw, prof = {"c2": (4096, 1, 8191, "flat"), "c3": (1 << 18, 1, 511, "flat"),
                     "c4": (32, 16, 524288, "pointer")}[cfg]
codec = capnproto_amd.Codec(0)
L = codec.lib
L.cpk_debug_stamps.argtypes = [C.c_int, C.POINTER(C.c_uint64)]
off, total = codec.gen_offsets(n, nseg=nseg, seg_words=sw, seed=20261015)
words = codec.gen_messages(prof, off, total, nseg=nseg, seed=20261015)
codec.timing(True)
for rep in range(3):
    out = (C.c_uint64 * 16)()
    L.cpk_debug_stamps(0, out)
    codec.timing_read_all()
    packed, moff, st = codec.pack_messages(words, off)
    codec.sync()
    L.cpk_debug_stamps(0, out)
    tm = codec.timing_read_all()
print(cfg, "pack kernel ms (stamps build):", round(tm["pack"][0], 4))
waves = out[15] or 1  # acc[15] = 1 per (persistent) wave
print("wave lifetime us:", round(out[14] / waves / 100, 2))
names = ["loads issue", "classes (+load wait)", "look-ahead", "cover/publish exit", "entry wait",
         "bytes+publish agg", "finish prev: flush + positions", "emission", "tail",
         "finish prev: look-back"]
tot = sum(out[i] for i in range(10))
print("cycles/wave", round(tot / waves))
for i, nm in enumerate(names):
    print(f"  {nm:32s} {out[i] / waves:12.0f}  {100 * out[i] / max(tot, 1):5.1f}%")
ntiles = (int(off[-1].item()) + 1023) // 1024
print("tiles", ntiles, "look-backs past the group per tile", round(out[10] / ntiles, 3),
      "group windows per tile", round(out[11] / ntiles, 3),
      "in-group hop cycles/tile", round(out[12] / ntiles), "group hop cycles/tile", round(out[13] / ntiles))
