import sys, time, json
sys.argv = ["bench.py"]
sys.path.insert(0, ".")
import torch, bench, capnproto_amd
codec = capnproto_amd.Codec(0)
off, total = codec.gen_offsets(4096, nseg=1, seg_words=8191, seed=20261015)
words = codec.gen_messages("flat", off, total, nseg=1, seed=20261015)
packed, moff, st = codec.pack_messages(words, off); codec.sync()
cs = [codec] + [capnproto_amd.Codec(0) for _ in range(3)]
for ns in (2, 3, 4):
    for ch in (8, 12, 16, 24):
        r = bench.host_inclusive_pipelined(cs[:ns], words, off, total, 4096, moff, 5, chunks=ch)
        print("streams", ns, "chunks", ch, r["GiBps"], r["ms_per_step"], r["round_trip_exact"])
