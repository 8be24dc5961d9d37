"""The reference API (include/cpk_capnp.h: writePackedMessage, PackedMessageReader,
PackedFdMessageReader, _::PackedOutputStream, computeUnpackedSizeInWords) on the MI355X codec:
tests/facade_test.cpp restates serialize-packed-test.c++ against the façade with the
reference's fixtures (tests/golden)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "capnproto_amd", "cpk_facade_test")
STREAM_BIN = os.path.join(ROOT, "capnproto_amd", "cpk_stream_test")
GOLDEN = os.path.join(ROOT, "tests", "golden")


@pytest.mark.gpu
def test_facade_reference_api_on_gpu():
    assert os.path.exists(BIN), "build with make -C capnproto_amd"
    r = subprocess.run([BIN, GOLDEN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout


def test_facade_refuses_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    if not os.path.exists(BIN):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "capnproto_amd")])
    r = subprocess.run([BIN, GOLDEN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "no HIP device" in r.stderr, r.stdout + r.stderr


@pytest.mark.gpu
def test_packed_message_stream_on_gpu():
    """PackedMessageStream (serialize-async.h:42-133 with packed framing): socket pairs and
    pipes, batched writes, EOF and premature-EOF rules (tests/stream_test.cpp)."""
    assert os.path.exists(STREAM_BIN), "build with make -C capnproto_amd"
    r = subprocess.run([STREAM_BIN, GOLDEN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout


def test_stream_refuses_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    if not os.path.exists(STREAM_BIN):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "capnproto_amd")])
    r = subprocess.run([STREAM_BIN, GOLDEN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "no HIP device" in r.stderr, r.stdout + r.stderr
