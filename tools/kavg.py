#!/usr/bin/env python3
"""Per-kernel average durations (us) from rocprofv3 kernel_stats CSVs: kavg.py CSV [LABEL]."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = {}
for r in rows:
    n = r["Name"].replace("(anonymous namespace)::", "")
    n = n.split("(")[0].split("::")[-1]
    if any(k in n for k in ("unpack", "pack_", "header", "message_bits", "flat_", "split", "meet", "walk")):
        out[n[:28]] = round(float(r["AverageNs"]) / 1e3, 1)
print(sys.argv[2] if len(sys.argv) > 2 else "", out)
