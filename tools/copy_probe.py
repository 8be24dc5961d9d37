#!/usr/bin/env python3
"""The bench's device-to-device copy ceiling alone (bench.measure_copy): our copy kernel's sweep
and the runtime's own copy.    python3 tools/copy_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import capnproto_amd  # noqa: E402

codec = capnproto_amd.Codec(0)
best, sweep = bench.measure_copy(codec)
print(json.dumps({"best_GBps": round(best, 1), "sweep": sweep}))
