#!/usr/bin/env python3
"""Per-kernel average durations (us) of the codec kernels in rocprofv3 kernel_stats CSVs:
    python3 tools/kstats.py gpurun_out/TAG_*  (directories holding *kernel_stats.csv)"""
import csv
import glob
import sys

for d in sys.argv[1:]:
    fs = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)
    if not fs:
        continue
    out = []
    for r in csv.DictReader(open(fs[0])):
        n = r["Name"]
        if "cpk::" not in n or "copy_kernel" in n or "gen_" in n or "fill_kernel" in n:
            continue
        short = n.replace("void ", "").replace("cpk::(anonymous namespace)::", "").split("(")[0]
        out.append(f"{short}={float(r['AverageNs']) / 1e3:.1f}")
    print(d.rstrip("/").split("/")[-1], " ".join(out))
