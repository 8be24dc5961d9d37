"""cpk-convert: `capnp convert` between binary / packed / flat / flat-packed on the device codec
(compiler/capnp.c++:773-800, :1027-1134).

The golden-file cases are the reference's own CLI tests (capnp-test.sh:69-70: binary:packed and
packed:binary over testdata) plus the same fixtures through the flat formats, which hold for
messages already in the canonical single-segment layout (testdata flat == binary minus its
table).  Multi-message streams and a random batch are checked against the CPU oracle; a truncated
stream must write the messages before the damage and fail with the reference's message.
"""
import os
import subprocess

import numpy as np
import pytest

import cases
import pyoracle as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "capnproto_amd", "cpk-convert")
G = os.path.join(ROOT, "tests", "golden")


def golden(name: str) -> bytes:
    with open(os.path.join(G, name), "rb") as f:
        return f.read()


def convert(spec: str, data: bytes):
    r = subprocess.run([BIN, spec], input=data, capture_output=True, timeout=120)
    return r.returncode, r.stdout, r.stderr.decode(errors="replace")


def ok(spec: str, data: bytes) -> bytes:
    rc, out, err = convert(spec, data)
    assert rc == 0, f"{spec}: rc {rc}: {err}"
    return out


@pytest.mark.gpu
@pytest.mark.parametrize(
    "spec,src,want",
    [
        ("binary:packed", "binary", "packed"),  # capnp-test.sh:69
        ("packed:binary", "packed", "binary"),  # capnp-test.sh:70
        ("binary:packed", "segmented", "segmented-packed"),
        ("packed:binary", "segmented-packed", "segmented"),
        ("flat:flat-packed", "flat", "packedflat"),
        ("flat-packed:flat", "packedflat", "flat"),
        ("binary:flat", "binary", "flat"),
        ("flat:binary", "flat", "binary"),
        ("packed:flat-packed", "packed", "packedflat"),
        ("flat-packed:packed", "packedflat", "packed"),
        ("binary:packed", "addressbook.bin", "addressbook.packed"),
        ("packed:binary", "addressbook.packed", "addressbook.bin"),
        ("binary:binary", "segmented", "segmented"),
        ("packed:packed", "segmented-packed", "segmented-packed"),
    ],
)
def test_convert_fixtures(spec, src, want):
    assert ok(spec, golden(src)) == golden(want)


@pytest.mark.gpu
def test_convert_message_stream():
    """Several messages on stdin, converted one after another (capnp.c++:795-797)."""
    names = ["binary", "segmented", "addressbook.bin", "binary", "addressbook.bin"]
    packed = {"binary": "packed", "segmented": "segmented-packed",
              "addressbook.bin": "addressbook.packed"}
    src = b"".join(golden(n) for n in names)
    want = b"".join(golden(packed[n]) for n in names)
    assert ok("binary:packed", src) == want
    assert ok("packed:binary", want) == src


@pytest.mark.gpu
def test_convert_random_batch_matches_oracle():
    rng = np.random.default_rng(44)
    words, off = cases.message_batch(rng, 300, max_seg=6, max_words=900)
    oracle = P.Oracle()
    packed, _, status = oracle.pack_batch(words, off)
    assert (status == 0).all()
    assert ok("binary:packed", words.tobytes()) == packed.tobytes()
    assert ok("packed:binary", packed.tobytes()) == words.tobytes()


@pytest.mark.gpu
def test_convert_empty_input():
    for spec in ("binary:packed", "packed:binary"):
        assert ok(spec, b"") == b""


@pytest.mark.gpu
def test_convert_truncated_stream():
    a, b = golden("packed"), golden("segmented-packed")
    rc, out, err = convert("packed:binary", a + b[: len(b) // 2])
    assert rc == 1
    assert out == golden("binary")  # the message before the damage is written
    assert "ERROR CONVERTING PREVIOUS MESSAGE" in err
    assert "Premature end of packed input." in err


@pytest.mark.gpu
def test_convert_refuses_relayout():
    rc, out, err = convert("binary:flat", golden("segmented"))
    assert rc == 1 and out == b"" and "several segments" in err


def test_convert_usage_without_gpu():
    """Argument errors are reported before any device call."""
    if not os.path.exists(BIN):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "capnproto_amd")])
    for args in ([], ["binary"], ["binary:json"], ["a:b", "c:d"]):
        r = subprocess.run([BIN] + args, input=b"", capture_output=True, timeout=60)
        assert r.returncode == 2, args
