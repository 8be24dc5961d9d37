"""PCIe probe for the host-inclusive path: pinned H2D, D2H, and both at once on two streams
(256 MiB each), then the pipelined host-inclusive C2 round trip for a few stream/chunk counts.
Run once per copy-engine setting (e.g. HSA_ENABLE_SDMA=0 for shader copies)."""
import os, sys, time
sys.argv = ["bench.py"]
sys.path.insert(0, ".")
import torch, bench, capnproto_amd

n = 256 << 20
h1 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
h2 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
d1 = torch.empty(n, dtype=torch.uint8, device="cuda")
d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, reps=5):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps): fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def both():
    with torch.cuda.stream(s1): d1.copy_(h1, non_blocking=True)
    with torch.cuda.stream(s2): h2.copy_(d2, non_blocking=True)


sdma = os.environ.get("HSA_ENABLE_SDMA", "default")
print("SDMA", sdma, "H2D GB/s %.1f" % (n / timed(lambda: d1.copy_(h1, non_blocking=True)) / 1e9),
      "D2H GB/s %.1f" % (n / timed(lambda: h2.copy_(d2, non_blocking=True)) / 1e9),
      "both GB/s %.1f" % (2 * n / timed(both) / 1e9), flush=True)
codec = capnproto_amd.Codec(0)
off, total = codec.gen_offsets(4096, nseg=1, seg_words=8191, seed=20261015)
words = codec.gen_messages("flat", off, total, nseg=1, seed=20261015)
packed, moff, st = codec.pack_messages(words, off); codec.sync()
cs = [codec] + [capnproto_amd.Codec(0) for _ in range(3)]
for ns, ch in ((2, 8), (2, 16), (4, 16), (4, 32)):
    r = bench.host_inclusive_pipelined(cs[:ns], words, off, total, 4096, moff, 5, chunks=ch)
    print("SDMA", sdma, "streams", ns, "chunks", ch, r["GiBps"], r["ms_per_step"], r["round_trip_exact"], flush=True)
