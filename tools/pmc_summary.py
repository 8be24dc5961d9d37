#!/usr/bin/env python3
"""Per-kernel averages of the rocprofv3 counter passes written by tools/gpu_pmc3.sh, and the HBM
traffic per launch of each tile kernel (gpurun_out/TAG_traffic_CFG.json, the file bench.py's
roofline.traffic reads once copied to profiles/traffic_CFG.json).

HBM bytes: FETCH_SIZE and WRITE_SIZE are kilobytes; on gfx950 FETCH_SIZE counts half the bytes of
wide (16 B/lane) streaming reads, so it is doubled (MI355X_MICROARCH.md, HBM/rocprofv3 section).
The doubling is exact only for that access width: other widths are uncalibrated."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out_dir, tag, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
# the kernels of the timed step (pack + unpack); the generator's size scan and fills
# (scan_kernel, fill_kernel, gen_kernel: the bench's input setup) and torch's kernels are not
KERNELS = {"unpack_tiles_kernel": "unpack_tiles", "header_kernel": "unpack_header",
           "message_bits_kernel": "pack_framing", "chunk_bits_kernel": "pack_framing"}


def short(name):
    if "cpk::" not in name:
        return None
    if "unpack_tiles_kernel<false, 1>" in name:
        return "unpack_index"
    if "unpack_tiles_kernel<false, 2>" in name:
        return "unpack_expand"
    if "unpack_resolve_kernel" in name:
        return "unpack_resolve"
    if "pack_tile_kernel" in name:
        return "pack_tile"
    if "pack_place_kernel" in name:
        return "pack_place"
    for k, v in KERNELS.items():
        if k in name:
            return v
    return None


vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(out_dir, f"{tag}_p*", "**", "*counter_collection.csv"),
                          recursive=True)):
    per = defaultdict(float)  # (dispatch, kernel, counter) -> summed over dims
    for row in csv.DictReader(open(f)):
        k = short(row.get("Kernel_Name", ""))
        if not k:
            continue
        key = (row.get("Dispatch_Id"), k, row.get("Counter_Name"))
        per[key] += float(row.get("Counter_Value", 0) or 0)
    for (disp, k, c), v in per.items():
        vals[k][c].append(v)

traffic = {}
for k in sorted(vals):
    avg = {c: sum(v) / len(v) for c, v in vals[k].items() if v}
    print(f"== {k}")
    for c in sorted(avg):
        print(f"   {c:24s} {avg[c]:16.1f}")
    waves = avg.get("SQ_WAVES")
    if waves:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                  "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM"):
            if c in avg:
                print(f"   per wave {c:15s} {avg[c] / waves:12.1f}")
    if "SQ_WAVE_CYCLES" in avg and "SQ_BUSY_CYCLES" in avg:
        print(f"   wave-cycles / busy-cycles {avg['SQ_WAVE_CYCLES'] / max(avg['SQ_BUSY_CYCLES'], 1):.1f}")
    if "FETCH_SIZE" in avg or "WRITE_SIZE" in avg:
        rd = 2 * 1024 * avg.get("FETCH_SIZE", 0.0)
        wr = 1024 * avg.get("WRITE_SIZE", 0.0)
        traffic[k] = {"read_bytes": round(rd), "write_bytes": round(wr), "bytes": round(rd + wr),
                      "note": "rocprofv3 FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, per launch"}
        print(f"   HBM traffic per launch: read {rd / 1e6:.1f} MB  write {wr / 1e6:.1f} MB")
# the pack "launch" the bench times is tile + place; per-step HBM bytes of every kernel
pk = [k for k in ("pack_tile", "pack_place") if k in traffic]
if pk:
    traffic["pack"] = {f: sum(traffic[k][f] for k in pk) for f in ("read_bytes", "write_bytes",
                                                                   "bytes")}
    traffic["pack"]["note"] = "pack_tile + pack_place (the bench's pack timer), per launch"
traffic["step_total_bytes"] = sum(v["bytes"] for k, v in traffic.items()
                                  if isinstance(v, dict) and k != "pack")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402  (kernel_source_hash: pins the file to the kernels it measured)

traffic["kernel_src_sha256"] = bench.kernel_source_hash()
json.dump(traffic, open(os.path.join(out_dir, f"{tag}_traffic_{cfg}.json"), "w"), indent=1)
