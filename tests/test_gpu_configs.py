"""GPU parity for every BASELINE.json configuration at full size, pinned to the reference.

* C1 -- the addressbook sample (samples/addressbook.c++:47-79): tests/golden/addressbook.bin is
  the 288-byte message the sample writes, addressbook.packed the 151 bytes the reference packs it
  to (both hash-pinned to the compiled sample in SURVEY.md 8(c); tools/make_addressbook.py).
* C2-C5 -- the bench workloads, regenerated on the device, packed, hashed and compared with
  tests/golden/manifest.json: SHA-256 of the reference's packed bytes for the same messages
  (tools/make_manifest.py packs them with oracle/_ref, i.e. capnp::writePackedMessage itself).
  Unpack is checked bit-exact against the generated input, with every status OK at the default
  traversal limit (C4's messages are exactly 8 Mi words, the limit, accepted by the reference's
  `<=` at serialize.c++:235).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import pyoracle as P
from gpu_util import dev, host_u64

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
MAN = json.load(open(os.path.join(G, "manifest.json")))["configs"]


@pytest.fixture(scope="module")
def codec():
    import capnproto_amd

    c = capnproto_amd.Codec(0)
    yield c
    c.close()


def sha_dev(t, chunk=1 << 28):
    """SHA-256 of a device tensor's bytes (copied to the host in pieces)."""
    import torch

    b = t.view(torch.uint8) if t.dtype != torch.uint8 else t
    h = hashlib.sha256()
    for i in range(0, b.numel(), chunk):
        h.update(memoryview(b[i : i + chunk].cpu().numpy()))
    return h.hexdigest()


def test_c1_addressbook_round_trip(codec):
    msg = open(os.path.join(G, "addressbook.bin"), "rb").read()
    ref = open(os.path.join(G, "addressbook.packed"), "rb").read()
    assert len(msg) == 288 and len(ref) == 151
    w = np.frombuffer(msg, "<u8")
    words = dev(codec, w)
    off = dev(codec, np.array([0, len(w)], np.int64))
    packed, moff, st = codec.pack_messages(words, off)
    codec.sync()
    assert st.cpu().numpy().tolist() == [0]
    n = int(moff[-1].item())
    assert packed[:n].cpu().numpy().tobytes() == ref
    back, woff, ust = codec.unpack_messages(dev(codec, np.frombuffer(ref, np.uint8)),
                                            dev(codec, np.array([0, len(ref)], np.int64)),
                                            len(w), nbytes=len(ref))
    codec.sync()
    assert ust.cpu().numpy().tolist() == [0]
    assert host_u64(back[: len(w)]).tobytes() == msg


def test_generator_matches_host_restatement(codec):
    """The device generator and the oracle's host copy build the same words (what pins the
    manifests, computed on the host, to the device-generated bench inputs)."""
    ora = P.Oracle()
    for name in ("c2", "c3", "c4", "c5", "c5r0of8"):
        c = MAN[name]
        k = min(c["nmsgs"], 3 if name == "c4" else 300)
        off, total = codec.gen_offsets(k, nseg=c["nseg"], seg_words=c["seg_words"], seed=c["seed"],
                                       first_msg=c["first_msg"], msg_stride=c["msg_stride"])
        words = codec.gen_messages(c["profile"], off, total, nseg=c["nseg"], seed=c["seed"],
                                   first_msg=c["first_msg"], msg_stride=c["msg_stride"])
        hoff = ora.gen_offsets(k, nseg=c["nseg"], seg_words=c["seg_words"], seed=c["seed"],
                               first_msg=c["first_msg"], msg_stride=c["msg_stride"])
        hw = ora.gen_messages(c["profile"], hoff, nseg=c["nseg"], seed=c["seed"],
                              first_msg=c["first_msg"], msg_stride=c["msg_stride"])
        assert (off.cpu().numpy().view(np.uint64) == hoff).all(), name
        assert host_u64(words[:total]).tobytes() == hw.tobytes(), name


def run_config(codec, name, prefix=False, limit=None):
    c = MAN[name]
    ref = c["prefix"] if prefix else c
    n = ref["nmsgs"]
    off, total = codec.gen_offsets(n, nseg=c["nseg"], seg_words=c["seg_words"], seed=c["seed"],
                                   first_msg=c["first_msg"], msg_stride=c["msg_stride"])
    assert total == ref["words"]
    words = codec.gen_messages(c["profile"], off, total, nseg=c["nseg"], seed=c["seed"],
                               first_msg=c["first_msg"], msg_stride=c["msg_stride"])
    packed, moff, st = codec.pack_messages(words, off)
    codec.sync()
    assert int((st != 0).sum().item()) == 0
    Pb = int(moff[-1].item())
    assert Pb == ref["packed_bytes"]
    assert sha_dev(packed[:Pb]) == ref["sha256_packed"], f"{name}: packed bytes != reference"
    assert sha_dev(moff) == ref["sha256_out_off"], f"{name}: packed offsets != reference"
    back, woff, ust = codec.unpack_messages(packed, moff, total, nbytes=Pb,
                                            traversal_limit_words=limit)
    codec.sync()
    return words, back, woff, ust, off, total


C5_SHARDS = [f"c5r{r}of8" for r in range(8)]  # the 8-GPU round-robin shards of C5


@pytest.mark.parametrize("name,prefix", [("c2", False), ("c3", True), ("c3", False),
                                         ("c4", True), ("c5", True)] +
                         [(s, True) for s in C5_SHARDS])
def test_config_pack_matches_reference_and_round_trips(codec, name, prefix):
    words, back, woff, ust, off, total = run_config(codec, name, prefix)
    assert int((ust != 0).sum().item()) == 0
    assert bool((woff == off).all().item())
    import torch

    assert torch.equal(back[:total], words[:total])


@pytest.mark.slow
@pytest.mark.parametrize("name", ["c4", "c5"] + C5_SHARDS)
def test_config_full_size(codec, name):
    """Full C4 (256 x 64 MiB at exactly the 8 Mi-word traversal limit, 16 GiB), full C5 (its
    first 4 Mi messages) and every one of the eight round-robin shards of the 8-GPU C5 run (4 Mi
    mixed messages each, about 14 GiB): packed bytes hashed against the reference's."""
    import torch

    words, back, woff, ust, off, total = run_config(codec, name)
    assert int((ust != 0).sum().item()) == 0
    assert bool((woff == off).all().item())
    assert torch.equal(back[:total], words[:total])
    del words, back
    torch.cuda.empty_cache()


def test_c4_traversal_limit_edges(codec):
    """C4 messages hold exactly 8 Mi words: accepted at the default limit (serialize.c++:235
    `totalWords <= limit`), rejected one word below it."""
    c = MAN["c4"]
    n = 2
    off, total = codec.gen_offsets(n, nseg=c["nseg"], seg_words=c["seg_words"], seed=c["seed"])
    words = codec.gen_messages(c["profile"], off, total, nseg=c["nseg"], seed=c["seed"])
    packed, moff, st = codec.pack_messages(words, off)
    codec.sync()
    Pb = int(moff[-1].item())
    for limit, want in ((8 << 20, 0), ((8 << 20) - 1, P.MESSAGE_TOO_LARGE)):
        _, _, ust = codec.unpack_messages(packed, moff, total, nbytes=Pb,
                                          traversal_limit_words=limit)
        codec.sync()
        assert ust.cpu().numpy().tolist() == [want] * n, limit


@pytest.mark.slow
def test_c4_geometric_stretches_match_oracle(codec):
    """C4's shape with SURVEY 8(d)'s geometric zero stretches (mean 300 words; the bench's
    `c4g` line, capnproto_amd/workloads.py): stretches far shorter and far longer than the
    generator's 264-336 words, most crossing the 256-word run cap.  No manifest describes these
    words, so the device's packed bytes and offsets for the whole 16 GiB batch are compared with
    the oracle's on a host copy, and the round trip is exact."""
    import torch

    from capnproto_amd.workloads import geometric_stretches, zero_stretches

    c = MAN["c4"]
    n = c["nmsgs"]
    off, total = codec.gen_offsets(n, nseg=c["nseg"], seg_words=c["seg_words"], seed=c["seed"])
    words = codec.gen_messages(c["profile"], off, total, nseg=c["nseg"], seed=c["seed"])
    geometric_stretches(words, off, c["nseg"], seed=c["seed"])
    packed, moff, st = codec.pack_messages(words, off)
    codec.sync()
    assert int((st != 0).sum().item()) == 0
    Pb = int(moff[-1].item())
    hw = host_u64(words[:total])
    zs = zero_stretches(hw[9 : 9 + (8 << 20)])  # message 0's body
    assert 280 < zs.mean() < 320 and (zs < 264).mean() > 0.4 and (zs > 336).mean() > 0.25
    ref, roff, rst = P.Oracle().pack_batch(hw, off.cpu().numpy().view(np.uint64))
    assert (rst == 0).all() and len(ref) == Pb
    assert (moff.cpu().numpy().view(np.uint64) == roff).all()
    assert np.array_equal(packed[:Pb].cpu().numpy(), ref), "packed bytes != oracle"
    del ref, hw
    back, woff, ust = codec.unpack_messages(packed, moff, total, nbytes=Pb)
    codec.sync()
    assert int((ust != 0).sum().item()) == 0
    assert bool((woff == off).all().item())
    assert torch.equal(back[:total], words[:total])
    del words, back
    torch.cuda.empty_cache()
