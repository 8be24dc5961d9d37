"""The bench's reshaped C4 input (capnproto_amd/workloads.py) on the CPU: geometric zero
stretches of mean 300 words around 4-76-word pointer / small-int runs, segment tables untouched,
reproducible per seed, and an exact round trip through the oracle (the GPU comparison is
tests/test_gpu_configs.py::test_c4_geometric_stretches_match_oracle)."""
import numpy as np
import torch

import pyoracle as P
from capnproto_amd.workloads import geometric_stretches, zero_stretches


def batch(n=4, seg_words=65536, seed=3):
    o = P.Oracle()
    hoff = o.gen_offsets(n, nseg=16, seg_words=seg_words, seed=seed)
    hw = o.gen_messages("pointer", hoff, nseg=16, seed=seed)
    return o, hoff, hw


def test_stretches_tables_and_round_trip():
    o, hoff, hw = batch()
    table = [hw[int(a) : int(a) + 9].copy() for a in hoff[:-1]]
    w = torch.from_numpy(hw.view(np.int64))  # shares hw's memory
    geometric_stretches(w, torch.from_numpy(hoff.view(np.int64).copy()), 16, seed=11)
    for a, t in zip(hoff[:-1], table):
        assert (hw[int(a) : int(a) + 9] == t).all()
    zs = np.concatenate([zero_stretches(hw[int(a) + 9 : int(b)]) for a, b in zip(hoff, hoff[1:])])
    assert 270 < zs.mean() < 330
    assert (zs > 256).mean() > 0.35 and (zs < 264).mean() > 0.4 and (zs > 336).mean() > 0.25
    assert zs.max() > 1000 and zs.min() < 10
    pk, poff, st = o.pack_batch(hw, hoff)
    back, woff, ust = o.unpack_batch(pk, poff, len(hw))
    assert (st == 0).all() and (ust == 0).all()
    assert (woff == hoff).all() and np.array_equal(back, hw)


def test_reproducible_per_message_seed():
    _, hoff, hw = batch(n=3, seg_words=4096)
    a = torch.from_numpy(hw.view(np.int64).copy())
    b = a.clone()
    off = torch.from_numpy(hoff.view(np.int64).copy())
    geometric_stretches(a, off, 16, seed=5)
    geometric_stretches(b, off, 16, seed=5)
    assert torch.equal(a, b)
    # message i is seeded by its global id: a shard starting at message 1 rebuilds message 1
    c = a.clone()
    sub = off[1:3] - off[1]
    geometric_stretches(c[int(off[1]) : int(off[2])], sub, 16, seed=5, first_msg=1)
    assert torch.equal(c, a)
