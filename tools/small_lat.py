#!/usr/bin/env python3
"""Small-message latency of the host entry points alone (bench.py's small_message_latency):
    python tools/small_lat.py [REPS]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import capnproto_amd  # noqa: E402

codec = capnproto_amd.Codec(0)
print(json.dumps(bench.small_message_latency(codec, int(sys.argv[1]) if len(sys.argv) > 1 else 300)))
