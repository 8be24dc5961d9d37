"""Helpers for the GPU parity tests (numpy <-> device tensors, batch builders)."""
from __future__ import annotations

import numpy as np


def dev(codec, arr, dtype=None):
    import torch

    a = np.ascontiguousarray(arr)
    if a.dtype == np.uint64 or a.dtype == np.dtype("<u8"):
        a = a.view(np.int64)
    t = torch.from_numpy(a.copy() if a.size else np.zeros(1, a.dtype))
    if dtype is not None:
        t = t.to(dtype)
    t = t.to(codec.device)
    return t if a.size else t[:0]


def host_u64(t) -> np.ndarray:
    return t.cpu().numpy().view(np.uint64)


def host_u8(t) -> np.ndarray:
    return t.cpu().numpy().astype(np.uint8, copy=False)


def offsets(lengths) -> np.ndarray:
    off = np.zeros(len(lengths) + 1, np.int64)
    off[1:] = np.cumsum(lengths)
    return off


def concat_bytes(chunks):
    b = b"".join(chunks)
    return np.frombuffer(b, np.uint8).copy() if b else np.zeros(0, np.uint8), offsets(
        [len(c) for c in chunks])
