#!/usr/bin/env python3
"""Diagnostic: per-call latency of the host entry points on the addressbook sample (as the bench's
small_message_latency), for rocprofv3 --kernel-trace --memory-copy-trace: the kernels and copies of
each call and the gaps between them."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import capnproto_amd  # noqa: E402
from bench import small_message_latency  # noqa: E402

codec = capnproto_amd.Codec(0)
r = small_message_latency(codec, reps=int(sys.argv[1]) if len(sys.argv) > 1 else 200)
print(r)
t0 = time.perf_counter()
codec.sync()
print("sync us", round(1e6 * (time.perf_counter() - t0), 1))
