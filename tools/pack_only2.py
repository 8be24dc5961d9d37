"""Pack-only timing loop for profiling (rocprofv3 --kernel-trace --stats)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capnproto_amd  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
n, nseg, sw, prof = {"c2": (4096, 1, 8191, "flat"), "c3": (1 << 18, 1, 511, "flat"),
                     "c4": (32, 16, 524288, "pointer")}[cfg]
codec = capnproto_amd.Codec(0)
off, total = codec.gen_offsets(n, nseg=nseg, seg_words=sw, seed=20261015)
words = codec.gen_messages(prof, off, total, nseg=nseg, seed=20261015)
packed, moff, st = codec.pack_messages(words, off)
for _ in range(10):
    codec.pack_messages(words, off, out=packed, msg_out_off=moff, status=st)
codec.sync()
print("ok", int(moff[-1].item()))
