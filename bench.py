#!/usr/bin/env python3
"""bench.py -- device-resident packed encode+decode throughput on MI355X.

Metric (BASELINE.json): "packed encode+decode GiB/s (device-resident), 4 KiB-64 MiB msg batch".
One step = writePackedMessage over every message of the rank's batch (cpk_pack_messages) followed
by PackedMessageReader over the packed result (cpk_unpack_messages), both on HBM-resident
buffers.  value = unpacked bytes of all ranks / wall time of one step (max over ranks).

    python bench.py [--config c2|c3|c4|c5] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N        (independent shards, weak scaling)

Extra JSON objects: "roofline" (dominant kernel, timed live with HIP events on its stream) and
"cpu_baseline" (the reference CPU codec -- oracle/_ref, compiled from the reference's sources --
timed on a bounded sample of the same workload on this host, 1 thread, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

# SURVEY.md 8(d) configurations.  seg_words=0: per-message size 2^k words, k uniform in [3, 11].
CONFIGS = {
    "c2": dict(nmsgs=4096, nseg=1, seg_words=8191, profile="flat",
               workload="C2: 4096 x 64 KiB flat-struct messages (1 table word + 8191 words)"),
    "c3": dict(nmsgs=1 << 20, nseg=1, seg_words=511, profile="flat",
               workload="C3: 1 Mi x 4 KiB flat-struct messages (tag-byte dominated)"),
    "c4": dict(nmsgs=256, nseg=16, seg_words=524288, profile="pointer",
               workload="C4: 256 x 64 MiB pointer-heavy messages, 16 segments each"),
    "c5": dict(nmsgs=(32 << 20) // 8, nseg=1, seg_words=0, profile="mixed", shard="round_robin",
               workload="C5: 32 Mi mixed-size messages (64 B-16 KiB), round-robin, 4 Mi per GPU"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="CPU-baseline budget (bounded sample of the same workload)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-inclusive", action="store_true",
                    help="also time the H2D/D2H-inclusive path (reported on stderr)")
    return ap.parse_args()


def cpu_baseline(words_np, off_np, seconds):
    """The reference codec (oracle/_ref: capnproto serialize-packed.c++ compiled from its own
    sources) or, if that build is absent, the C restatement -- on a bounded sample."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as P

    try:
        impl, kind = P.Reference(), "reference"
        pack = lambda: impl.pack_batch(words_np, off_np)  # noqa: E731
    except OSError:
        impl, kind = P.Oracle(), "port"
        pack = lambda: impl.pack_batch(words_np, off_np)[:2]  # noqa: E731
    packed, poff = pack()
    packed = np.ascontiguousarray(packed)
    cap = len(words_np)

    def unpack():
        return impl.unpack_batch(packed, poff, cap)

    U = words_np.nbytes
    tp = tu = 0.0
    reps = 0
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end or reps == 0:
        t0 = time.perf_counter()
        pack()
        t1 = time.perf_counter()
        unpack()
        t2 = time.perf_counter()
        tp += t1 - t0
        tu += t2 - t1
        reps += 1
    return {
        "value": U * reps / (tp + tu) / 2**30,
        "unit": "GiB/s",
        "cores": 1,
        "kind": kind,
        "sample": f"{len(off_np) - 1} messages ({U / 2**20:.1f} MiB unpacked, "
                  f"{len(packed) / 2**20:.2f} MiB packed) x {reps} pack+unpack passes, 1 thread",
        "pack_GiBps": U * reps / tp / 2**30,
        "unpack_GiBps": U * reps / tu / 2**30,
    }, packed, poff


def main():
    args = parse()
    import numpy as np
    import torch

    import capnproto_amd
    from capnproto_amd.shard import reduce_step, shard_messages

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus and rank == 0:
        print(f"note: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier():
        if dist is not None:
            dist.barrier()

    cfg = CONFIGS[args.config]
    codec = capnproto_amd.Codec(local)
    # Independent message shards (weak scaling: nmsgs per GPU): capnproto_amd/shard.py.
    first, stride, n = shard_messages(rank, world, cfg["nmsgs"] * world, cfg.get("shard", "block"))
    off, total = codec.gen_offsets(n, nseg=cfg["nseg"], seg_words=cfg["seg_words"],
                                   seed=args.seed, first_msg=first, msg_stride=stride)
    words = codec.gen_messages(cfg["profile"], off, total, nseg=cfg["nseg"], seed=args.seed,
                               first_msg=first, msg_stride=stride)
    cap = codec.packed_bound(total, n * (cfg["nseg"] + 1)) + 64
    packed = torch.empty(cap, dtype=torch.uint8, device=codec.device)
    moff = torch.empty(n + 1, dtype=torch.int64, device=codec.device)
    pst = torch.empty(n, dtype=torch.int32, device=codec.device)
    back = torch.empty(total, dtype=torch.int64, device=codec.device)
    woff = torch.empty(n + 1, dtype=torch.int64, device=codec.device)
    ust = torch.empty(n, dtype=torch.int32, device=codec.device)
    codec.reserve(total, cap, n)

    # packed size is a function of the input: learn it once (the caller's framing knows it)
    codec.pack_messages(words, off, out=packed, msg_out_off=moff, status=pst)
    codec.sync()
    P = int(moff[-1].item())
    U = total * 8

    def step():
        codec.pack_messages(words, off, out=packed, msg_out_off=moff, status=pst)
        codec.unpack_messages(packed, moff, total, nbytes=P, words=back, msg_word_off=woff,
                              status=ust)

    for _ in range(args.warmup):
        step()
    codec.sync()
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    codec.sync()
    dt = t1 - t0

    # correctness of what was timed: exact round trip + statuses
    ok = bool((pst == 0).all().item() and (ust == 0).all().item() and torch.equal(woff, off)
              and torch.equal(back, words[:total]))

    # per-kernel durations: a second pass of the same steps with HIP events around every tile
    # kernel, on the stream the kernels run on (kept out of the wall-clock pass above)
    codec.timing_read_all()  # discard
    codec.timing(True)
    for _ in range(args.steps):
        step()
    codec.timing(False)
    codec.sync()
    kt = codec.timing_read_all()
    kms = {k: (v[0] / v[1] if v[1] else 0.0) for k, v in kt.items()}

    red = reduce_step(dt, float(U), float(P), kms["pack"], kms["unpack"], ok,
                      dist=dist, device=codec.device)
    dt_max, U_all = red["dt_max"], red["unpacked_all"]
    ok_all = red["ok_all"]

    result = None
    if rank == 0:
        ms_per_step = dt_max / args.steps * 1e3
        value = U_all / (dt_max / args.steps) / 2**30
        # algorithmic HBM bytes of one launch of each tile kernel
        algo = {"pack_count": U, "pack_emit": U + P, "unpack_index": P, "unpack_expand": U + P}
        if kms["pack_count"] == 0:  # single-pass pack kernel (CPK_PACK_FUSED=1)
            algo = {"pack": U + P, "unpack_index": P, "unpack_expand": U + P}
        kern = {k: {"ms": round(kms[k], 4),
                    "GBps": round(algo[k] / (kms[k] * 1e-3) / 1e9, 1) if kms[k] > 0 else None,
                    "algorithmic_bytes": int(algo[k])} for k in algo}
        for k in ("pack", "unpack_resolve", "unpack_fallback"):
            kern.setdefault(k, {"ms": round(kms[k], 4)})
        dom = max(algo, key=lambda k: kms[k])
        dom_ms = kms[dom]
        achieved = algo[dom] / (dom_ms * 1e-3) / 1e9
        rt_ms = kms["pack"] + kms["unpack"]
        rt = 2.0 * (U + P) / (rt_ms * 1e-3) / 1e9
        traffic = None
        tf = os.path.join(ROOT, "profiles", f"traffic_{args.config}.json")
        if os.path.exists(tf):
            try:
                t = json.load(open(tf)).get(dom)
                traffic = int(t["bytes"]) if isinstance(t, dict) else t
            except Exception:
                traffic = None
        result = {
            "metric": "packed encode+decode GiB/s (device-resident), 4 KiB-64 MiB msg batch",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (deterministic on-device generator, SURVEY.md 8(d))",
            "config": {
                "workload": cfg["workload"],
                "messages_per_gpu": n,
                "unpacked_bytes_per_gpu": U,
                "packed_bytes_per_gpu": P,
                "packed_ratio": round(P / U, 4),
                "profile": cfg["profile"],
                "parallelism": f"dp{world} (independent message shards, no data-path collective)",
            },
            "parity": "bit-exact round trip" if ok_all else "MISMATCH",
            "roofline": {
                "bound": "hbm",
                "kernel": dom,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": int(algo[dom]),
                "kernels": kern,
                "pack_ms": round(kms["pack"], 4),
                "unpack_ms": round(kms["unpack"], 4),
                "roundtrip_GBps": round(rt, 1),
                "roundtrip_frac": round(rt / HBM_PEAK_GBS, 4),
            },
            "cpu_baseline": None,
        }

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        k = min(n, max(1, (4 << 20) // max(1, U // n)))  # ~4 MiB sample of the same workload
        o = off[: k + 1].cpu().numpy().astype(np.uint64)
        wsample = words[: int(o[-1])].cpu().numpy().view(np.uint64)
        cb, ref_packed, ref_off = cpu_baseline(wsample, o, args.cpu_seconds)
        result["cpu_baseline"] = cb
        # packed bytes of the sample must equal the reference's bit for bit
        gp = packed[: int(moff[k].item())].cpu().numpy()
        if gp.tobytes() != np.asarray(ref_packed).tobytes():
            result["parity"] = "MISMATCH vs reference packed bytes"
        else:
            result["parity"] += f"; packed bytes == {cb['kind']} CPU codec on the sample"

    if args.host_inclusive and world == 1:
        hi = host_inclusive(codec, words, off, total, n, cap, args.steps)
        print(json.dumps({"host_inclusive": hi}), file=sys.stderr)

    if rank == 0:
        print(json.dumps(result))
    codec.close()
    if dist is not None:
        dist.destroy_process_group()


def host_inclusive(codec, words, off, total, n, cap, steps):
    """U / (H2D(U) + pack + D2H(P) + H2D(P) + unpack + D2H(U)) with pinned host buffers."""
    import torch

    hw = torch.empty(total, dtype=torch.int64, pin_memory=True)
    hw.copy_(words[:total])
    hp = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
    hb = torch.empty(total, dtype=torch.int64, pin_memory=True)
    dw = torch.empty_like(words[:total])
    dp = torch.empty(cap, dtype=torch.uint8, device=codec.device)
    dp2 = torch.empty(cap, dtype=torch.uint8, device=codec.device)
    moff = torch.empty(n + 1, dtype=torch.int64, device=codec.device)
    back = torch.empty(total, dtype=torch.int64, device=codec.device)
    codec.pack_messages(words, off, out=dp, msg_out_off=moff)
    codec.sync()
    P = int(moff[-1].item())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        dw.copy_(hw, non_blocking=True)
        codec.pack_messages(dw, off, out=dp, msg_out_off=moff)
        hp[:P].copy_(dp[:P], non_blocking=True)
        dp2[:P].copy_(hp[:P], non_blocking=True)
        codec.unpack_messages(dp2, moff, total, nbytes=P, words=back)
        hb.copy_(back, non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return {"GiBps": total * 8 / dt / 2**30, "ms_per_step": dt * 1e3,
            "path": "pinned H2D(U) + pack + D2H(P) + H2D(P) + unpack + D2H(U)"}


if __name__ == "__main__":
    main()
