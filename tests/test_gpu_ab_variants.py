"""The library's measured alternative kernels, each selected by an environment variable the library
reads once per process (bench.py KERNEL_ENV), run through the parity suite of its
direction in a child process with the variable set:

* CPK_UNPACK_SPLIT=1 -- the split message decode (index, resolve and expand launches;
  cpk_unpack.hip "Split decode") through tests/test_gpu_unpack.py: reference fixtures, error
  cases, locked chains that gate the expansion launch onto the look-back, the UINT_MAX segment
  count;
* CPK_FLAT_SPLIT=0 -- the stream split's one-pass flat decode (the default decodes the flat
  stream in two launches) through tests/test_gpu_stream.py: the oracle's message boundaries on
  random, text and edge-case streams, truncated and corrupted ones, the UINT_MAX segment count."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("knob,value,suite", [("CPK_UNPACK_SPLIT", "1", "test_gpu_unpack.py"),
                                              ("CPK_FLAT_SPLIT", "0", "test_gpu_stream.py")])
def test_suite_through_variant(knob, value, suite):
    env = dict(os.environ, **{knob: value})
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        "--timeout", "120", "--timeout-method", "thread",
                        os.path.join(HERE, suite)],
                       env=env, capture_output=True, text=True, timeout=400, cwd=HERE)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert " passed" in r.stdout
