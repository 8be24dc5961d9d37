"""capnproto_amd -- MI355X-native Cap'n Proto packed wire codec.

The product is ``libcpk_hip.so`` (C ABI: include/cpk.h) with hand-written gfx950 HIP kernels for
pack (serialize-packed.c++:307-431) and unpack (:34-183).  This module is a thin ctypes host layer
over that ABI for Python callers (tests, bench): device buffers are torch tensors on ``cuda:N``
(PyTorch is plumbing here -- allocation and streams), the kernels are ours.

There is no CPU fallback: importing works anywhere, but constructing a ``Codec`` without the
built library or without a GPU raises.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libcpk_hip.so")

# include/cpk.h cpk_status
OK = 0
PREMATURE_EOF = 1
RUN_OVERSHOOT = 2
TOO_MANY_SEGMENTS = 3
MESSAGE_TOO_LARGE = 4
INVALID_PACKED = 5
BAD_FRAMING = 6
TRAILING_BYTES = 7
CAPACITY = 8
INVALID_ARGUMENT = 9
HIP_ERROR = 10
EMPTY_MESSAGE = 11
INTERNAL = 12
NO_DEVICE = 13

PROFILES = {"flat": 0, "pointer": 1, "text": 2, "mixed": 3}

_lib = None


class CpkError(RuntimeError):
    def __init__(self, status: int, where: str = ""):
        self.status = status
        msg = load_library().cpk_status_string(status).decode()
        super().__init__(f"{where}: cpk status {status}: {msg}" if where else msg)


def build(force: bool = False) -> str:
    """Compile libcpk_hip.so for gfx950 with hipcc (make -C capnproto_amd)."""
    import subprocess

    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", HERE, "-j8"])
    return LIB_PATH


def load_library():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(f"{LIB_PATH} is missing: build it with `make -C capnproto_amd` "
                      "(there is no CPU fallback)")
    L = C.CDLL(LIB_PATH)
    vp, u64, i32, u32 = C.c_void_p, C.c_uint64, C.c_int32, C.c_uint32
    sigs = {
        "cpk_status_string": (C.c_char_p, [i32]),
        "cpk_abi_version": (C.c_int, []),
        "cpk_init": (C.c_int, [C.c_int, C.POINTER(vp)]),
        "cpk_destroy": (C.c_int, [vp]),
        "cpk_reserve": (C.c_int, [vp, u64, u64, u64]),
        "cpk_sync": (C.c_int, [vp, vp]),
        "cpk_copy_ranges": (C.c_int, [vp, vp, vp, vp, vp, u64, vp, vp]),
        "cpk_packed_bound": (u64, [u64, u64]),
        "cpk_pack_chunks": (C.c_int, [vp, vp, u64, vp, u64, vp, u64, vp, vp]),
        "cpk_pack_messages": (C.c_int, [vp, vp, u64, vp, u64, vp, u64, vp, vp, vp]),
        "cpk_unpack_messages": (C.c_int, [vp, vp, u64, vp, u64, vp, u64, vp, vp, vp, vp]),
        "cpk_unpacked_size": (C.c_int, [vp, vp, u64, vp, u64, vp, vp, vp]),
        "cpk_unpack_chunks": (C.c_int, [vp, vp, u64, vp, vp, u64, vp, u64, vp, vp]),
        "cpk_pack_segments": (C.c_int, [vp, vp, vp, u64, vp, u64, vp, vp]),
        "cpk_split_packed_stream": (C.c_int, [vp, vp, u64, vp, u64, u64, vp, vp, vp, vp, vp,
                                              vp]),
        "cpk_pack_messages_host": (C.c_int, [vp, vp, u64, vp, u64, vp, u64, vp, vp]),
        "cpk_unpack_messages_host": (C.c_int, [vp, vp, u64, vp, u64, vp, u64, vp, vp, vp]),
        "cpk_gen_messages": (C.c_int, [vp, C.c_int, u64, u64, u64, u64, u32, vp, vp, vp]),
        "cpk_gen_offsets": (C.c_int, [vp, u64, u64, u64, u64, u32, u64, vp, C.POINTER(u64), vp]),
        "cpk_timing_enable": (C.c_int, [vp, C.c_int]),
        "cpk_timing_read": (C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(u64),
                                      C.POINTER(C.c_double), C.POINTER(u64)]),
        "cpk_timing_read_all": (C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(u64)]),
        "cpk_debug_copy": (C.c_int, [vp, vp, u64, u32, vp]),
    }
    for name, (res, args) in sigs.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


class Limits(C.Structure):
    _fields_ = [("traversal_limit_words", C.c_uint64)]


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


class Codec:
    """One cpk_ctx on one GPU.  All tensors are device tensors; words are int64 (bit patterns of
    little-endian u64 words), packed bytes uint8, offsets int64, statuses int32."""

    def __init__(self, device: int = 0):
        import torch

        self.torch = torch
        self.lib = load_library()
        if not torch.cuda.is_available():
            raise CpkError(NO_DEVICE, "Codec")
        self.device = torch.device("cuda", device)
        h = C.c_void_p()
        self._check(self.lib.cpk_init(device, C.byref(h)), "cpk_init")
        self.ctx = h

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.cpk_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _check(st, where):
        if st != OK:
            raise CpkError(st, where)

    def _stream(self, stream):
        s = stream if stream is not None else self.torch.cuda.current_stream(self.device)
        return C.c_void_p(s.cuda_stream)

    def sync(self, stream=None):
        self._check(self.lib.cpk_sync(self.ctx, self._stream(stream)), "cpk_sync")

    def copy_ranges(self, src, src_off, dst_off, length, dst, stream=None):
        """dst[dst_off[i] : +length[i]] = src[src_off[i] : +length[i]] for every i (device u8
        tensors, int64 offset / length tensors of one size; include/cpk.h cpk_copy_ranges)."""
        n = src_off.numel()
        if dst_off.numel() != n or length.numel() != n:
            raise ValueError("copy_ranges: offset and length tensors differ in size")
        self._check(self.lib.cpk_copy_ranges(self.ctx, _ptr(src), _ptr(src_off), _ptr(dst_off),
                                             _ptr(length), n, _ptr(dst), self._stream(stream)),
                    "cpk_copy_ranges")
        return dst

    def reserve(self, max_words, max_packed_bytes, max_items):
        self._check(self.lib.cpk_reserve(self.ctx, max_words, max_packed_bytes, max_items),
                    "cpk_reserve")

    def packed_bound(self, words: int, chunks: int) -> int:
        return int(self.lib.cpk_packed_bound(words, chunks))

    # ------------------------------------------------------------------ pack
    def pack_messages(self, words, msg_word_off, out=None, msg_out_off=None, status=None,
                      stream=None):
        """writePackedMessage for a batch of flat messages (see include/cpk.h)."""
        torch = self.torch
        n = msg_word_off.numel() - 1
        N = words.numel()
        if out is None:
            out = torch.empty(self.packed_bound(N, 2 * n + 1) + 16, dtype=torch.uint8,
                              device=self.device)
        if msg_out_off is None:
            msg_out_off = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        if status is None:
            status = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        self._check(self.lib.cpk_pack_messages(self.ctx, _ptr(words), N, _ptr(msg_word_off), n,
                                               _ptr(out), out.numel(), _ptr(msg_out_off),
                                               _ptr(status), self._stream(stream)),
                    "cpk_pack_messages")
        return out, msg_out_off, status[:n]

    def pack_chunks(self, words, chunk_word_off, out=None, chunk_out_off=None, stream=None):
        torch = self.torch
        n = chunk_word_off.numel() - 1
        N = words.numel()
        if out is None:
            out = torch.empty(self.packed_bound(N, n + 1) + 16, dtype=torch.uint8,
                              device=self.device)
        if chunk_out_off is None:
            chunk_out_off = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        self._check(self.lib.cpk_pack_chunks(self.ctx, _ptr(words), N, _ptr(chunk_word_off), n,
                                             _ptr(out), out.numel(), _ptr(chunk_out_off),
                                             self._stream(stream)), "cpk_pack_chunks")
        return out, chunk_out_off

    def pack_segments(self, segments, out=None, stream=None):
        """writePackedMessage over a list of device segments (int64 tensors, any addresses):
        no host gather (include/cpk.h cpk_pack_segments).  Returns (out, nbytes tensor)."""
        torch = self.torch
        n = len(segments)
        ptrs = (C.c_uint64 * max(n, 1))(*[s.data_ptr() for s in segments])
        sizes = (C.c_uint64 * max(n, 1))(*[s.numel() for s in segments])
        total = n // 2 + 1 + sum(s.numel() for s in segments)
        if out is None:
            out = torch.empty(self.packed_bound(total, n + 1) + 16, dtype=torch.uint8,
                              device=self.device)
        nbytes = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._check(self.lib.cpk_pack_segments(self.ctx, ptrs, sizes, n, _ptr(out), out.numel(),
                                               _ptr(nbytes), self._stream(stream)),
                    "cpk_pack_segments")
        return out, nbytes

    # ------------------------------------------------------------------ unpack
    def unpack_messages(self, packed, msg_in_off, words_capacity, nbytes=None, words=None,
                        msg_word_off=None, status=None, traversal_limit_words=None,
                        stream=None):
        """PackedMessageReader over a batch (see include/cpk.h)."""
        torch = self.torch
        n = msg_in_off.numel() - 1
        P = packed.numel() if nbytes is None else nbytes
        if words is None:
            words = torch.empty(max(words_capacity, 1), dtype=torch.int64, device=self.device)
        if msg_word_off is None:
            msg_word_off = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        if status is None:
            status = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        lim = None
        if traversal_limit_words is not None:
            lim = C.byref(Limits(traversal_limit_words))
        self._check(self.lib.cpk_unpack_messages(self.ctx, _ptr(packed), P, _ptr(msg_in_off), n,
                                                 _ptr(words), words_capacity, _ptr(msg_word_off),
                                                 _ptr(status), lim, self._stream(stream)),
                    "cpk_unpack_messages")
        return words, msg_word_off, status[:n]

    def unpacked_size(self, packed, in_off, nbytes=None, stream=None):
        torch = self.torch
        n = in_off.numel() - 1
        P = packed.numel() if nbytes is None else nbytes
        out = torch.empty(max(n, 1), dtype=torch.int64, device=self.device)
        status = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        self._check(self.lib.cpk_unpacked_size(self.ctx, _ptr(packed), P, _ptr(in_off), n,
                                               _ptr(out), _ptr(status), self._stream(stream)),
                    "cpk_unpacked_size")
        return out[:n], status[:n]

    def unpack_chunks(self, packed, in_off, word_off, words=None, nbytes=None, stream=None):
        torch = self.torch
        n = in_off.numel() - 1
        P = packed.numel() if nbytes is None else nbytes
        total = int(word_off[-1].item()) if n else 0
        if words is None:
            words = torch.empty(max(total, 1), dtype=torch.int64, device=self.device)
        status = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        self._check(self.lib.cpk_unpack_chunks(self.ctx, _ptr(packed), P, _ptr(in_off),
                                               _ptr(word_off), n, _ptr(words), words.numel(),
                                               _ptr(status), self._stream(stream)),
                    "cpk_unpack_chunks")
        return words, status[:n]

    def split_packed_stream(self, packed, words_capacity, max_msgs, nbytes=None, words=None,
                            traversal_limit_words=None, stream=None):
        """Stream boundary discovery (include/cpk.h cpk_split_packed_stream): messages back to
        back in one packed buffer, offsets unknown.  Returns (words, msg_word_off, msg_in_off,
        status, nmsgs) -- device tensors with max_msgs + 1 entries, nmsgs a 1-element device
        tensor."""
        torch = self.torch
        P = packed.numel() if nbytes is None else nbytes
        if words is None:
            words = torch.empty(max(words_capacity, 1), dtype=torch.int64, device=self.device)
        woff = torch.empty(max_msgs + 1, dtype=torch.int64, device=self.device)
        ioff = torch.empty(max_msgs + 1, dtype=torch.int64, device=self.device)
        status = torch.empty(max_msgs + 1, dtype=torch.int32, device=self.device)
        n = torch.empty(1, dtype=torch.int64, device=self.device)
        lim = None
        if traversal_limit_words is not None:
            lim = C.byref(Limits(traversal_limit_words))
        self._check(self.lib.cpk_split_packed_stream(self.ctx, _ptr(packed), P, _ptr(words),
                                                     words_capacity, max_msgs, _ptr(woff),
                                                     _ptr(ioff), _ptr(status), _ptr(n), lim,
                                                     self._stream(stream)),
                    "cpk_split_packed_stream")
        return words, woff, ioff, status, n

    # ------------------------------------------------------------------ measurement hooks
    def timing(self, on: bool = True):
        self._check(self.lib.cpk_timing_enable(self.ctx, 1 if on else 0), "cpk_timing_enable")

    def timing_read(self):
        """(pack_ms, pack_launches, unpack_ms, unpack_launches) since the last read."""
        pm, um = C.c_double(0), C.c_double(0)
        pl, ul = C.c_uint64(0), C.c_uint64(0)
        self._check(self.lib.cpk_timing_read(self.ctx, C.byref(pm), C.byref(pl), C.byref(um),
                                             C.byref(ul)), "cpk_timing_read")
        return pm.value, pl.value, um.value, ul.value

    TIMERS = ("pack", "unpack", "unpack_tiles", "unpack_fallback", "t4", "t5", "t6", "t7")

    def timing_read_all(self):
        """{timer name: (summed ms, launches)} since the last read (include/cpk.h timers)."""
        ms = (C.c_double * len(self.TIMERS))()
        n = (C.c_uint64 * len(self.TIMERS))()
        self._check(self.lib.cpk_timing_read_all(self.ctx, ms, n), "cpk_timing_read_all")
        return {k: (ms[i], n[i]) for i, k in enumerate(self.TIMERS)}

    # ------------------------------------------------------------------ synthetic workloads
    def gen_offsets(self, nmsgs, nseg=1, seg_words=0, seed=0, first_msg=0, msg_stride=1,
                    stream=None):
        off = self.torch.empty(nmsgs + 1, dtype=self.torch.int64, device=self.device)
        total = C.c_uint64(0)
        self._check(self.lib.cpk_gen_offsets(self.ctx, seed, first_msg, msg_stride, nmsgs, nseg,
                                             seg_words,
                                             _ptr(off), C.byref(total), self._stream(stream)),
                    "cpk_gen_offsets")
        return off, int(total.value)

    def gen_messages(self, profile, msg_word_off, total_words, nseg=1, seed=0, first_msg=0,
                     msg_stride=1, words=None, stream=None):
        if isinstance(profile, str):
            profile = PROFILES[profile]
        n = msg_word_off.numel() - 1
        if words is None:
            words = self.torch.empty(max(total_words, 1), dtype=self.torch.int64,
                                     device=self.device)
        self._check(self.lib.cpk_gen_messages(self.ctx, profile, seed, first_msg, msg_stride, n, nseg,
                                              _ptr(msg_word_off), _ptr(words),
                                              self._stream(stream)), "cpk_gen_messages")
        return words
