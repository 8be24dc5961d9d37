"""ctypes bindings for the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Two checkers live under oracle/:

* ``Oracle``    -- oracle/build/libcpk_oracle.so, our C restatement of the reference packed codec
                   (cpk_oracle.c; each function cites the reference file:line it restates).
* ``Reference`` -- oracle/_ref/libcpk_ref.so, the REAL reference codec (capnproto
                   c++/src/capnp/serialize-packed.c++, serialize.c++, kj/io.c++) compiled from
                   /root/reference by oracle/Makefile.ref behind our own C shim (ref_shim.c++).
                   Present only where it was built (this container, and the GPU box when the
                   prebuilt .so travels with the snapshot).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product (capnproto_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "build", "libcpk_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "libcpk_ref.so")

# include/cpk.h cpk_status
OK, PREMATURE_EOF, RUN_OVERSHOOT, TOO_MANY_SEGMENTS, MESSAGE_TOO_LARGE = 0, 1, 2, 3, 4
INVALID_PACKED, BAD_FRAMING, TRAILING_BYTES, CAPACITY = 5, 6, 7, 8
DEFAULT_TRAVERSAL_LIMIT = 8 * 1024 * 1024  # capnp/message.h:54

_u8p = C.POINTER(C.c_uint8)
_u64p = C.POINTER(C.c_uint64)
_i32p = C.POINTER(C.c_int32)
_szp = C.POINTER(C.c_size_t)


def _ptr(a: np.ndarray, t):
    return a.ctypes.data_as(t)


def build_oracle() -> None:
    subprocess.check_call(["make", "-s", "-C", HERE])


def words_of(b: bytes) -> np.ndarray:
    assert len(b) % 8 == 0
    return np.frombuffer(b, dtype="<u8").copy()


def packed_bound(words: int, chunks: int) -> int:
    return words * 8 + (words + 1) // 2 + 2 * chunks + 16


def split_flat(words: np.ndarray):
    """Segments of a flat message (table + segments, serialize.c++:161-190 layout)."""
    t32 = words[: max(1, len(words))].view("<u4")
    nseg = int(t32[0]) + 1
    tw = nseg // 2 + 1
    sizes = [int(x) for x in words[:tw].view("<u4")[1 : nseg + 1]]
    segs, pos = [], tw
    for s in sizes:
        segs.append(words[pos : pos + s])
        pos += s
    assert pos == len(words), "inconsistent flat message"
    return segs


def flat_from_segments(segs) -> np.ndarray:
    """serializeSegmentTable + segments (serialize.c++:311-330)."""
    nseg = len(segs)
    tw = nseg // 2 + 1
    table = np.zeros(tw * 2, dtype="<u4")
    table[0] = nseg - 1
    for i, s in enumerate(segs):
        table[i + 1] = len(s)
    parts = [table.view("<u8")] + [np.asarray(s, dtype="<u8") for s in segs]
    return np.concatenate(parts) if parts else np.zeros(0, "<u8")


class Oracle:
    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build_oracle()
        L = self.lib = C.CDLL(path)
        L.cpko_pack_chunk.restype = C.c_size_t
        L.cpko_pack_chunk.argtypes = [_u64p, C.c_size_t, _u8p]
        L.cpko_pack_flat_message.restype = C.c_size_t
        L.cpko_pack_flat_message.argtypes = [_u64p, C.c_size_t, _u8p, _i32p]
        L.cpko_read_message.restype = C.c_int32
        L.cpko_read_message.argtypes = [_u8p, C.c_size_t, C.c_uint64, _u64p, C.c_size_t, _szp, _szp]
        L.cpko_unpack_exact.restype = C.c_int32
        L.cpko_unpack_exact.argtypes = [_u8p, C.c_size_t, _szp, _u64p, C.c_size_t]
        L.cpko_skip_words.restype = C.c_int32
        L.cpko_skip_words.argtypes = [_u8p, C.c_size_t, _szp, C.c_size_t]
        L.cpko_unpacked_size.restype = C.c_int32
        L.cpko_unpacked_size.argtypes = [_u8p, C.c_size_t, _u64p]
        L.cpko_pack_batch.restype = C.c_int32
        L.cpko_pack_batch.argtypes = [_u64p, _u64p, C.c_uint64, _u8p, _u64p, _i32p]
        L.cpko_unpack_batch.restype = C.c_int32
        L.cpko_unpack_batch.argtypes = [_u8p, _u64p, C.c_uint64, _u64p, C.c_uint64, _u64p, _i32p,
                                        C.c_uint64]
        L.cpko_splitmix64.restype = C.c_uint64
        L.cpko_splitmix64.argtypes = [C.c_uint64]
        L.cpko_gen_offsets.restype = None
        L.cpko_gen_offsets.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                       C.c_uint32, C.c_uint64, _u64p]
        L.cpko_gen_messages.restype = None
        L.cpko_gen_messages.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                        C.c_uint32, _u64p, _u64p]

    # -- host restatement of the bench generator (capnproto_amd/csrc/cpk_gen.hip)
    PROFILES = {"flat": 0, "pointer": 1, "text": 2, "mixed": 3}

    def gen_offsets(self, nmsgs, nseg=1, seg_words=0, seed=0, first_msg=0, msg_stride=1):
        off = np.zeros(nmsgs + 1, "<u8")
        self.lib.cpko_gen_offsets(seed, first_msg, msg_stride, nmsgs, nseg, seg_words,
                                  _ptr(off, _u64p))
        return off

    def gen_messages(self, profile, off, nseg=1, seed=0, first_msg=0, msg_stride=1):
        """Messages first_msg + i * msg_stride for i < len(off) - 1 (off may start anywhere)."""
        off = np.ascontiguousarray(off, dtype="<u8")
        words = np.zeros(max(1, int(off[-1] - off[0])), "<u8")
        self.lib.cpko_gen_messages(self.PROFILES.get(profile, profile), seed, first_msg,
                                   msg_stride, len(off) - 1, nseg, _ptr(off, _u64p),
                                   _ptr(words, _u64p))
        return words[: int(off[-1] - off[0])]

    # -- a1: PackedOutputStream::write(one piece)
    def pack_chunk(self, words) -> bytes:
        w = np.ascontiguousarray(words, dtype="<u8")
        out = np.zeros(packed_bound(len(w), 1), np.uint8)
        n = self.lib.cpko_pack_chunk(_ptr(w, _u64p), len(w), _ptr(out, _u8p))
        return out[:n].tobytes()

    # -- a5/a7: writePackedMessage over a flat message
    def pack_flat(self, words):
        w = np.ascontiguousarray(words, dtype="<u8")
        out = np.zeros(packed_bound(len(w), 600), np.uint8)
        st = C.c_int32(0)
        n = self.lib.cpko_pack_flat_message(_ptr(w, _u64p), len(w), _ptr(out, _u8p), C.byref(st))
        return out[:n].tobytes(), st.value

    # -- a2/a8: PackedMessageReader over an array; returns (status, flat words, consumed)
    def read_message(self, packed: bytes, limit: int = DEFAULT_TRAVERSAL_LIMIT, cap_words=None):
        b = np.frombuffer(packed, np.uint8).copy() if packed else np.zeros(1, np.uint8)
        if cap_words is None:
            cap_words = 300 + 8 * max(1, len(packed))
        out = np.zeros(cap_words, "<u8")
        consumed, nw = C.c_size_t(0), C.c_size_t(0)
        st = self.lib.cpko_read_message(_ptr(b, _u8p), len(packed), limit, _ptr(out, _u64p),
                                        cap_words, C.byref(consumed), C.byref(nw))
        return st, out[: nw.value].copy(), consumed.value

    def unpack_exact(self, packed: bytes, nwords: int):
        b = np.frombuffer(packed, np.uint8).copy() if packed else np.zeros(1, np.uint8)
        out = np.zeros(max(1, nwords), "<u8")
        pos = C.c_size_t(0)
        st = self.lib.cpko_unpack_exact(_ptr(b, _u8p), len(packed), C.byref(pos),
                                        _ptr(out, _u64p), nwords)
        return st, out[:nwords].copy(), pos.value

    def skip_words(self, packed: bytes, nwords: int):
        b = np.frombuffer(packed, np.uint8).copy() if packed else np.zeros(1, np.uint8)
        pos = C.c_size_t(0)
        st = self.lib.cpko_skip_words(_ptr(b, _u8p), len(packed), C.byref(pos), nwords)
        return st, pos.value

    def unpacked_size(self, packed: bytes):
        b = np.frombuffer(packed, np.uint8).copy() if packed else np.zeros(1, np.uint8)
        w = C.c_uint64(0)
        st = self.lib.cpko_unpacked_size(_ptr(b, _u8p), len(packed), C.byref(w))
        return st, w.value

    # -- batches (flat messages back to back)
    def pack_batch(self, words: np.ndarray, msg_word_off: np.ndarray):
        n = len(msg_word_off) - 1
        out = np.zeros(packed_bound(len(words), 2 * n + 600 * 0 + 2 * n), np.uint8)
        off = np.zeros(n + 1, "<u8")
        status = np.zeros(max(1, n), np.int32)
        self.lib.cpko_pack_batch(_ptr(words, _u64p), _ptr(msg_word_off, _u64p), n,
                                 _ptr(out, _u8p), _ptr(off, _u64p), _ptr(status, _i32p))
        return out[: int(off[n])], off, status[:n]

    def unpack_batch(self, packed: np.ndarray, msg_in_off: np.ndarray, words_cap: int,
                     limit: int = DEFAULT_TRAVERSAL_LIMIT):
        n = len(msg_in_off) - 1
        words = np.zeros(max(1, words_cap), "<u8")
        off = np.zeros(n + 1, "<u8")
        status = np.zeros(max(1, n), np.int32)
        p = packed if len(packed) else np.zeros(1, np.uint8)
        self.lib.cpko_unpack_batch(_ptr(p, _u8p), _ptr(msg_in_off, _u64p), n,
                                   _ptr(words, _u64p), words_cap, _ptr(off, _u64p),
                                   _ptr(status, _i32p), limit)
        return words[: int(off[n])], off, status[:n]


class Reference:
    """The real reference codec (oracle/_ref/libcpk_ref.so).  Raises OSError if not built."""

    def __init__(self, path: str = REF_SO):
        if not os.path.exists(path):
            raise OSError(f"reference build missing: {path} (make -f oracle/Makefile.ref)")
        L = self.lib = C.CDLL(path)
        L.ref_last_error.restype = C.c_char_p
        L.ref_pack_chunk.argtypes = [_u64p, C.c_uint64, _u8p, C.c_uint64, _u64p]
        L.ref_pack_segments.argtypes = [C.POINTER(_u64p), C.POINTER(C.c_uint32), C.c_uint32,
                                        _u8p, C.c_uint64, _u64p]
        L.ref_pack_segments_unbuffered.argtypes = L.ref_pack_segments.argtypes
        L.ref_read_message.argtypes = [_u8p, C.c_uint64, C.c_uint64, _u64p, C.c_uint64, _u64p,
                                       _u64p, C.POINTER(C.c_uint32)]
        L.ref_unpack_exact.argtypes = [_u8p, C.c_uint64, _u64p, C.c_uint64, _u64p]
        L.ref_skip_words.argtypes = [_u8p, C.c_uint64, C.c_uint64, _u64p]
        L.ref_unpacked_size.argtypes = [_u8p, C.c_uint64, _u64p]
        L.ref_pack_batch.argtypes = [_u64p, _u64p, C.c_uint64, _u8p, C.c_uint64, _u64p]
        L.ref_unpack_batch.argtypes = [_u8p, _u64p, C.c_uint64, _u64p, C.c_uint64, _u64p]
        for f in ("ref_pack_chunk", "ref_pack_segments", "ref_pack_segments_unbuffered",
                  "ref_read_message", "ref_unpack_exact", "ref_skip_words", "ref_unpacked_size",
                  "ref_pack_batch", "ref_unpack_batch"):
            getattr(L, f).restype = C.c_int

    def last_error(self) -> str:
        return self.lib.ref_last_error().decode(errors="replace")

    def pack_chunk(self, words) -> bytes:
        w = np.ascontiguousarray(words, dtype="<u8")
        if len(w) == 0:
            w = np.zeros(1, "<u8")
            nwords = 0
        else:
            nwords = len(w)
        cap = packed_bound(nwords, 1)
        out = np.zeros(cap, np.uint8)
        n = C.c_uint64(0)
        st = self.lib.ref_pack_chunk(_ptr(w, _u64p), nwords, _ptr(out, _u8p), cap, C.byref(n))
        assert st == 0, self.last_error()
        return out[: n.value].tobytes()

    def pack_segments(self, segs, unbuffered: bool = False) -> bytes:
        keep = [np.ascontiguousarray(s, dtype="<u8") if len(s) else np.zeros(1, "<u8")
                for s in segs]
        ptrs = (_u64p * len(segs))(*[_ptr(k, _u64p) for k in keep])
        sizes = (C.c_uint32 * len(segs))(*[len(s) for s in segs])
        total = sum(len(s) for s in segs) + len(segs) // 2 + 1
        cap = packed_bound(total, len(segs) + 1)
        out = np.zeros(cap, np.uint8)
        n = C.c_uint64(0)
        f = self.lib.ref_pack_segments_unbuffered if unbuffered else self.lib.ref_pack_segments
        st = f(ptrs, sizes, len(segs), _ptr(out, _u8p), cap, C.byref(n))
        assert st == 0, self.last_error()
        return out[: n.value].tobytes()

    def read_message(self, packed: bytes, limit: int = DEFAULT_TRAVERSAL_LIMIT, cap_words=None):
        b = np.frombuffer(packed, np.uint8).copy() if packed else np.zeros(1, np.uint8)
        if cap_words is None:
            cap_words = 600 + 8 * max(1, len(packed))
        out = np.zeros(cap_words, "<u8")
        consumed, nw, nseg = C.c_uint64(0), C.c_uint64(0), C.c_uint32(0)
        st = self.lib.ref_read_message(_ptr(b, _u8p), len(packed), limit, _ptr(out, _u64p),
                                       cap_words, C.byref(consumed), C.byref(nw), C.byref(nseg))
        return st, out[: nw.value].copy(), consumed.value

    def unpack_exact(self, packed: bytes, nwords: int):
        b = np.frombuffer(packed, np.uint8).copy() if packed else np.zeros(1, np.uint8)
        out = np.zeros(max(1, nwords), "<u8")
        consumed = C.c_uint64(0)
        st = self.lib.ref_unpack_exact(_ptr(b, _u8p), len(packed), _ptr(out, _u64p), nwords,
                                       C.byref(consumed))
        return st, out[:nwords].copy(), consumed.value

    def skip_words(self, packed: bytes, nwords: int):
        b = np.frombuffer(packed, np.uint8).copy() if packed else np.zeros(1, np.uint8)
        consumed = C.c_uint64(0)
        st = self.lib.ref_skip_words(_ptr(b, _u8p), len(packed), nwords, C.byref(consumed))
        return st, consumed.value

    def unpacked_size(self, packed: bytes):
        b = np.frombuffer(packed, np.uint8).copy() if packed else np.zeros(1, np.uint8)
        w = C.c_uint64(0)
        st = self.lib.ref_unpacked_size(_ptr(b, _u8p), len(packed), C.byref(w))
        return st, w.value

    def pack_batch(self, words: np.ndarray, msg_word_off: np.ndarray):
        n = len(msg_word_off) - 1
        cap = packed_bound(len(words), 2 * n + 2)
        out = np.zeros(cap, np.uint8)
        off = np.zeros(n + 1, "<u8")
        st = self.lib.ref_pack_batch(_ptr(words, _u64p), _ptr(msg_word_off, _u64p), n,
                                     _ptr(out, _u8p), cap, _ptr(off, _u64p))
        assert st == 0, self.last_error()
        return out[: int(off[n])], off

    def unpack_batch(self, packed: np.ndarray, msg_in_off: np.ndarray, words_cap: int):
        n = len(msg_in_off) - 1
        words = np.zeros(max(1, words_cap), "<u8")
        off = np.zeros(n + 1, "<u8")
        st = self.lib.ref_unpack_batch(_ptr(packed, _u8p), _ptr(msg_in_off, _u64p), n,
                                       _ptr(words, _u64p), words_cap, _ptr(off, _u64p))
        assert st == 0, self.last_error()
        return words[: int(off[n])], off


def reference_available() -> bool:
    return os.path.exists(REF_SO)
