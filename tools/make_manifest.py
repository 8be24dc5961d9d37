#!/usr/bin/env python3
"""Pin the full-size bench configurations to the REAL reference codec: SHA-256 manifests.

For every configuration bench.py measures (C2-C5 of SURVEY.md 8(d)), the messages are rebuilt on
the host by the oracle's restatement of the device generator (cpk_gen.hip), packed message by
message with the reference itself (oracle/_ref/libcpk_ref.so: writePackedMessage over an
ArrayOutputStream, serialize-packed.c++:460-464), and hashed as one stream:

    sha256_packed      the concatenated packed bytes of the batch (what cpk_pack_messages writes)
    sha256_out_off     the n + 1 packed offsets, little-endian u64
    sha256_words       the concatenated flat messages (what cpk_unpack_messages must restore)

plus the same three for a short prefix of the batch (fast GPU tests).  Output:
tests/golden/manifest.json (data only: sizes and hashes).  Needs /root/reference built by
`make -f oracle/Makefile.ref`; run in the build container:

    python tools/make_manifest.py [c2 c3 c4 c5 c5r0of8 ...]
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), ROOT]
import pyoracle as P  # noqa: E402

SEED = 20261015  # bench.py --seed default
# name -> (nmsgs, nseg, seg_words, profile, first_msg, stride, prefix messages, batch)
CONFIGS = {
    "c2": (4096, 1, 8191, "flat", 0, 1, 64, 4096),
    "c3": (1 << 20, 1, 511, "flat", 0, 1, 4096, 65536),
    "c4": (256, 16, 524288, "pointer", 0, 1, 2, 1),
    "c5": ((32 << 20) // 8, 1, 0, "mixed", 0, 1, 65536, 262144),
    # rank 0 of the 8-GPU round-robin shard (bench.py --gpus 8: first_msg = rank, stride = 8)
    "c5r0of8": ((32 << 20) // 8, 1, 0, "mixed", 0, 8, 65536, 262144),
}
# ranks 1-7 of the same 8-GPU round-robin shard (first_msg = rank)
for _r in range(1, 8):
    CONFIGS[f"c5r{_r}of8"] = ((32 << 20) // 8, 1, 0, "mixed", _r, 8, 65536, 262144)
OUT = os.path.join(ROOT, "tests", "golden", "manifest.json")


def run(name, ora, ref):
    n, nseg, sw, prof, first, stride, npre, batch = CONFIGS[name]
    off_all = ora.gen_offsets(n, nseg=nseg, seg_words=sw, seed=SEED, first_msg=first,
                              msg_stride=stride)
    hp, ho, hw = hashlib.sha256(), hashlib.sha256(), hashlib.sha256()
    pre = None
    P_total = 0
    t0 = time.time()
    for b0 in range(0, n, batch):
        b1 = min(n, b0 + batch)
        off = off_all[b0 : b1 + 1]
        words = ora.gen_messages(prof, off, nseg=nseg, seed=SEED, first_msg=first + b0 * stride,
                                 msg_stride=stride)
        loff = (off - off[0]).astype("<u8")
        packed, poff = ref.pack_batch(words, loff)
        poff = poff.astype("<u8") + P_total
        hp.update(memoryview(np.ascontiguousarray(packed)))
        ho.update(memoryview(poff[:-1] if b1 < n else poff))
        hw.update(memoryview(words))
        if pre is None and b0 == 0:
            k = min(npre, b1)
            ph, po, pw = hashlib.sha256(), hashlib.sha256(), hashlib.sha256()
            pk = int(poff[k] - P_total)
            ph.update(memoryview(np.ascontiguousarray(packed[:pk])))
            po.update(memoryview(poff[: k + 1]))
            pw.update(memoryview(words[: int(loff[k])]))
            pre = {"nmsgs": k, "words": int(loff[k]), "packed_bytes": pk,
                   "sha256_packed": ph.hexdigest(), "sha256_out_off": po.hexdigest(),
                   "sha256_words": pw.hexdigest()}
        P_total += int(len(packed))
    U = int(off_all[-1]) * 8
    rec = {"nmsgs": n, "nseg": nseg, "seg_words": sw, "profile": prof, "first_msg": first,
           "msg_stride": stride, "seed": SEED, "words": int(off_all[-1]), "unpacked_bytes": U,
           "packed_bytes": P_total, "sha256_packed": hp.hexdigest(),
           "sha256_out_off": ho.hexdigest(), "sha256_words": hw.hexdigest(), "prefix": pre,
           "packed_by": "reference (oracle/_ref/libcpk_ref.so: capnp::writePackedMessage)"}
    print(f"{name}: U={U} P={P_total} ({time.time() - t0:.1f} s)", flush=True)
    return rec


def main():
    names = sys.argv[1:] or list(CONFIGS)
    ora, ref = P.Oracle(), P.Reference()
    man = json.load(open(OUT)) if os.path.exists(OUT) else {}
    man.setdefault("generator", "capnproto_amd/csrc/cpk_gen.hip (host restatement: "
                                "oracle/cpk_oracle.c cpko_gen_*)")
    man.setdefault("configs", {})
    for nm in names:
        rec = run(nm, ora, ref)
        man = json.load(open(OUT)) if os.path.exists(OUT) else man  # (another run may have added)
        man.setdefault("configs", {})[nm] = rec
        with open(OUT, "w") as f:
            json.dump(man, f, indent=1, sort_keys=True)
            f.write("\n")


if __name__ == "__main__":
    main()
