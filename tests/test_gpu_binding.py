"""Reference callers through the reference-side binding (integration/kj_binding.h), executed:
oracle/_ref/kj_binding_test links the reference's own kj / capnp objects (MessageReader, kj
streams, FlatArrayMessageReader) but NOT its serialize-packed.o, so every packed byte comes from
libcpk_hip.so.  It runs serialize-packed-test.c++:90-195's expectPacksTo over the KATs, the
reference fixtures through writePackedMessage / PackedMessageReader, and samples/addressbook.c++'s
writePackedMessageToFd -> PackedFdMessageReader -> getRoot flow (integration/kj_binding_test.c++).
The binary is built in the container (oracle/Makefile.ref, needs the reference headers) and
travels to the GPU box with the tree."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "kj_binding_test")


@pytest.mark.skipif(not os.path.exists(BIN), reason="oracle/_ref/kj_binding_test not built")
def test_reference_callers_through_binding():
    # the reference's own packed codec is not in the binary: its packed entry points resolve to
    # the binding (cpk_kj::) and the façade in libcpk_hip.so
    import re

    nm = subprocess.run(["nm", "-C", BIN], capture_output=True, text=True).stdout
    assert not re.search(r"\s(capnp::_::PackedOutputStream|capnp::_::PackedInputStream|"
                         r"capnp::writePackedMessage|capnp::PackedMessageReader)", nm)
    assert re.search(r"\sU cpk_capnp::_::PackedOutputStream::write", nm)
    ldd = subprocess.run(["ldd", BIN], capture_output=True, text=True).stdout
    assert "libcpk_hip.so" in ldd
    r = subprocess.run([BIN, os.path.join(ROOT, "tests", "golden")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "binding ok" in r.stdout and "addressbook" in r.stdout


ABIN = os.path.join(ROOT, "oracle", "_ref", "kj_async_binding_test")


@pytest.mark.skipif(not os.path.exists(ABIN), reason="oracle/_ref/kj_async_binding_test not built")
def test_async_message_stream_through_binding():
    # capnp::MessageStream (serialize-async.h:42-108) with packed framing on the reference's kj
    # event loop: cpk_kj::PackedMessageStream over an OS socket pair and an in-memory kj pipe,
    # wire bytes == the reference's packed fixtures (integration/kj_async_binding_test.c++)
    import re

    nm = subprocess.run(["nm", "-C", ABIN], capture_output=True, text=True).stdout
    assert not re.search(r"\s(capnp::_::PackedOutputStream|capnp::_::PackedInputStream|"
                         r"capnp::writePackedMessage|capnp::PackedMessageReader)", nm)
    assert re.search(r"\sU cpk_read_packed_message_host", nm)
    assert re.search(r"\sU cpk_pack_messages_host", nm)
    try:
        r = subprocess.run([ABIN, os.path.join(ROOT, "tests", "golden")], capture_output=True,
                           text=True, timeout=60)
    except subprocess.TimeoutExpired as e:  # name the step that did not finish
        err = e.stderr.decode() if isinstance(e.stderr, bytes) else (e.stderr or "")
        pytest.fail("kj_async_binding_test timed out after:\n" + err[-2000:])
    assert r.returncode == 0, r.stderr[-3000:]
    assert "async binding ok" in r.stdout
