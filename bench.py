#!/usr/bin/env python3
"""bench.py -- device-resident packed encode+decode throughput on MI355X.

Metric (BASELINE.json): "packed encode+decode GiB/s (device-resident), 4 KiB-64 MiB msg batch".
One step = writePackedMessage over every message of the rank's batch (cpk_pack_messages) followed
by PackedMessageReader over the packed result (cpk_unpack_messages), both on HBM-resident
buffers.  value = unpacked bytes of all ranks / wall time of one step (max over ranks).

    python bench.py [--config c2|c3|c4|c5] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N        (independent shards, weak scaling)

The headline line is the --config workload (C2 by default).  At N=1 the default run also
measures C3 and C4 (``sub_results``, each with its own roofline), so one driver run covers the
4 KiB - 64 MiB range.  Every measured batch is checked after timing: exact device round trip,
and -- where tests/golden/manifest.json pins the workload -- SHA-256 of the packed bytes equal to
the reference codec's.  A mismatch (or a diagnostic build knob in the environment) prints no
``value`` and exits non-zero.

Extra JSON objects:
  roofline      headline: the round trip, 2(U+P) algorithmic bytes per step / wall time of a
                step, against the 8 TB/s HBM peak; plus the read-only fraction
                (U+P)/t, a D2D copy measured in the same run, and the dominant kernel alone
                (HIP events on the stream the kernels run on).
  cpu_baseline  the reference CPU codec (oracle/_ref, compiled from the reference's sources) on
                this host, 1 thread and all the host cores this job has, on a bounded sample of
                the same workload (rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "packed encode+decode GiB/s (device-resident), 4 KiB-64 MiB msg batch"

# SURVEY.md 8(d) configurations.  seg_words=0: per-message size 2^k words, k uniform in [3, 11].
CONFIGS = {
    "c2": dict(nmsgs=4096, nseg=1, seg_words=8191, profile="flat",
               workload="C2: 4096 x 64 KiB flat-struct messages (1 table word + 8191 words)"),
    "c3": dict(nmsgs=1 << 20, nseg=1, seg_words=511, profile="flat",
               workload="C3: 1 Mi x 4 KiB flat-struct messages (tag-byte dominated)"),
    "c4": dict(nmsgs=256, nseg=16, seg_words=524288, profile="pointer",
               workload="C4: 256 x 64 MiB pointer-heavy messages, 16 segments each"),
    # C4's shape with SURVEY 8(d)'s zero-stretch distribution (geometric, mean 300 words;
    # capnproto_amd/workloads.py) instead of the generator's 264-336-word stretches: an extra
    # line, not a headline config (no manifest: its packed bytes are checked against the oracle
    # in tests/test_gpu_configs.py, the round trip here)
    "c4g": dict(nmsgs=256, nseg=16, seg_words=524288, profile="pointer", stretches="geometric",
                workload="C4g: 256 x 64 MiB pointer-heavy messages, 16 segments each, "
                         "geometric zero stretches (mean 300 words)"),
    "c5": dict(nmsgs=(32 << 20) // 8, nseg=1, seg_words=0, profile="mixed", shard="round_robin",
               one_gpu_shard_of=8,
               workload="C5: 32 Mi mixed-size messages (64 B-16 KiB), round-robin, 4 Mi per GPU "
                        "(at N = 1: shard 0 of the 8-GPU run, messages 0, 8, 16, ...)"),
}
DEBUG_ENV = ("CPK_DEBUG_SKIP", "CPK_STAMPS")
# kernel-selection knobs (env): a headline number comes from the default kernels unless --ab is
# given.  The library's measured alternatives: CPK_UNPACK_SPLIT=1 the split
# message decode, CPK_FLAT_SPLIT=0 the one-pass flat decode of the stream split.  Every CPK_*
# variable that is set is recorded in the result's "kernels.knobs".
KERNEL_ENV: tuple = ("CPK_UNPACK_SPLIT", "CPK_FLAT_SPLIT")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--sub", default=None,
                    help="comma-separated extra configs measured after the headline "
                         "(default at N=1: c3,c4,c4g,c5; 'none' to skip)")
    ap.add_argument("--sub-steps", type=int, default=5)
    ap.add_argument("--shard", default=None, choices=["block", "round_robin", "bytes"],
                    help="message assignment to ranks (default: the config's)")
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="CPU-baseline budget (bounded sample of the same workload)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true",
                    help="time eager launches instead of the step captured as one HIP graph")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the manifest hash check (the device round trip is still checked)")
    ap.add_argument("--host-inclusive", action="store_true",
                    help="also time the serial (one stream) H2D/D2H-inclusive path")
    ap.add_argument("--no-split", action="store_true",
                    help="skip the stream-split (boundary discovery) measurement")
    ap.add_argument("--no-host", action="store_true",
                    help="skip the host-inclusive (pipelined) measurement")
    ap.add_argument("--ab", action="store_true",
                    help="allow non-default kernel-selection knobs (A/B runs; recorded in 'knobs')")
    return ap.parse_args()


def kernel_source_hash() -> str:
    """Content hash of the device code and of the host code that sequences its launches, carves
    its scratch and zeroes it (pins a committed PMC traffic file to what it measured)."""
    h = hashlib.sha256()
    for p in sorted(glob.glob(os.path.join(ROOT, "capnproto_amd", "csrc", "*.hip")) +
                    glob.glob(os.path.join(ROOT, "capnproto_amd", "csrc", "*.h")) +
                    glob.glob(os.path.join(ROOT, "capnproto_amd", "csrc", "*.cpp"))):
        h.update(os.path.basename(p).encode())
        h.update(open(p, "rb").read())
    return h.hexdigest()


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads() -> int:
    """Host cores this job may use: the box's CPU share (OMP_NUM_THREADS is set to it there),
    capped by what the machine reports."""
    n = os.cpu_count() or 1
    e = os.environ.get("OMP_NUM_THREADS")
    if e and e.isdigit() and int(e) > 0:
        n = min(n, int(e))
    return n


def cpu_baseline(sample_words, sample_off, seconds, threads):
    """The reference codec (oracle/_ref: capnproto serialize-packed.c++ compiled from its own
    sources) or, if that build is absent, the C restatement -- pack (ArrayOutputStream shape)
    then unpack (ArrayInputStream + PackedMessageReader shape) of a bounded sample, first on one
    thread, then on `threads` threads each owning a disjoint slice.  ctypes drops the GIL for
    the duration of each foreign call, so the threads run the codec in parallel."""
    import ctypes as C

    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as P

    try:
        impl, kind = P.Reference(), "reference"
    except OSError:
        impl, kind = P.Oracle(), "port"
    u8p, u64p, i32p = C.POINTER(C.c_uint8), C.POINTER(C.c_uint64), C.POINTER(C.c_int32)

    class Job:
        def __init__(self, words, off):
            self.words = np.ascontiguousarray(words, dtype="<u8")
            self.off = np.ascontiguousarray(off - off[0], dtype="<u8")
            self.n = len(off) - 1
            self.cap = P.packed_bound(len(self.words), 2 * self.n + 2)
            self.out = np.zeros(self.cap, np.uint8)
            self.poff = np.zeros(self.n + 1, "<u8")
            self.back = np.zeros(max(1, len(self.words)), "<u8")
            self.woff = np.zeros(self.n + 1, "<u8")
            self.st = np.zeros(max(1, self.n), np.int32)
            self.tp = self.tu = 0.0
            self.reps = 0

        def pack(self):
            if kind == "reference":
                impl.lib.ref_pack_batch(self.words.ctypes.data_as(u64p),
                                        self.off.ctypes.data_as(u64p), self.n,
                                        self.out.ctypes.data_as(u8p), self.cap,
                                        self.poff.ctypes.data_as(u64p))
            else:
                impl.lib.cpko_pack_batch(self.words.ctypes.data_as(u64p),
                                         self.off.ctypes.data_as(u64p), self.n,
                                         self.out.ctypes.data_as(u8p),
                                         self.poff.ctypes.data_as(u64p),
                                         self.st.ctypes.data_as(i32p))

        def unpack(self):
            if kind == "reference":
                impl.lib.ref_unpack_batch(self.out.ctypes.data_as(u8p),
                                          self.poff.ctypes.data_as(u64p), self.n,
                                          self.back.ctypes.data_as(u64p), len(self.back),
                                          self.woff.ctypes.data_as(u64p))
            else:
                impl.lib.cpko_unpack_batch(self.out.ctypes.data_as(u8p),
                                           self.poff.ctypes.data_as(u64p), self.n,
                                           self.back.ctypes.data_as(u64p), len(self.back),
                                           self.woff.ctypes.data_as(u64p),
                                           self.st.ctypes.data_as(i32p), 8 << 20)

        def run(self, t_end):
            while time.perf_counter() < t_end or self.reps == 0:
                t0 = time.perf_counter()
                self.pack()
                t1 = time.perf_counter()
                self.unpack()
                t2 = time.perf_counter()
                self.tp += t1 - t0
                self.tu += t2 - t1
                self.reps += 1

    # one thread on the first slice; then `threads` threads on slices of the whole sample
    nm = len(sample_off) - 1
    per = max(1, nm // threads)
    slices = [(i * per, min(nm, (i + 1) * per)) for i in range(threads) if i * per < nm]
    jobs = [Job(sample_words[int(sample_off[a]):int(sample_off[b])], sample_off[a:b + 1])
            for a, b in slices]
    jobs[0].pack()
    ref_packed = jobs[0].out[: int(jobs[0].poff[-1])].copy()
    one = jobs[0]
    one.run(time.perf_counter() + seconds / 2)
    U1 = one.words.nbytes
    single = {"value": U1 * one.reps / (one.tp + one.tu) / 2**30,
              "pack_GiBps": U1 * one.reps / one.tp / 2**30,
              "unpack_GiBps": U1 * one.reps / one.tu / 2**30, "cores": 1,
              "sample": f"{one.n} messages ({U1 / 2**20:.1f} MiB) x {one.reps} passes"}
    for j in jobs:
        j.tp = j.tu = 0.0
        j.reps = 0
    t_end = time.perf_counter() + seconds / 2
    w0 = time.perf_counter()
    th = [threading.Thread(target=j.run, args=(t_end,)) for j in jobs]
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - w0
    Ub = sum(j.words.nbytes * j.reps for j in jobs)
    multi = Ub / wall / 2**30
    return {
        "value": round(multi, 3),
        "unit": "GiB/s",
        "cores": len(jobs),
        "kind": kind,
        "sample": f"{nm} messages of the workload ({sample_words.nbytes / 2**20:.1f} MiB), "
                  f"{len(jobs)} threads each packing then unpacking its own slice for "
                  f"{seconds / 2:.0f} s; single-thread pass on {one.n} messages",
        "single_thread": {k: (round(v, 3) if isinstance(v, float) else v)
                          for k, v in single.items()},
        "nproc": os.cpu_count(),
        "cpu_model": cpu_model(),
    }, ref_packed, jobs[0].poff.copy(), one.n


def config_cpu_baseline(res, seconds):
    """cpu_baseline on a bounded sample of one measured config (rank 0, N = 1): ~4 MiB of its
    messages per host thread, copied from the device batch; also checks that the CPU codec's
    packed bytes of its first slice equal the device's.  Returns (baseline dict, same)."""
    import numpy as np

    words, off, packed, moff, total, cap = res["tensors"]
    nt = host_threads()
    per = max(1, (4 << 20) // max(1, res["U"] // res["n"]))  # ~4 MiB per thread
    k = min(res["n"], per * nt)
    o = off[: k + 1].cpu().numpy().astype(np.uint64)
    ws = words[: int(o[-1])].cpu().numpy().view(np.uint64)
    cb, ref_packed, ref_off, k1 = cpu_baseline(ws, o, seconds, nt)
    gp = packed[: int(moff[k1].item())].cpu().numpy()
    same = gp.tobytes() == np.asarray(ref_packed).tobytes()
    if not same:
        print(f"bench: {res['name']}: CPU codec packed bytes differ from the device's",
              file=sys.stderr)
    return cb, same


def measure_copy(codec, nbytes=1 << 31, reps=6):
    """Device-to-device copy ceiling in the same run: our streaming copy kernel (16 B per lane;
    capnproto_amd/csrc/cpk_stream.hip copy_kernel), the best of a sweep over 4 / 8 / 16 loads in
    flight per lane, default or non-temporal loads and stores, grid-strided or contiguous
    per-block shares, LDS-DMA staging (global_load_lds_dwordx4, 2 / 4 / 8 KiB per wave), and six
    grid sizes; read + write bytes / time of 2 GiB each way, timed with HIP events on the stream it
    runs on.  (MI355X_MICROARCH.md quotes 6.29 TB/s for a float4 copy.)"""
    import ctypes as C

    torch = codec.torch
    a = torch.empty(nbytes, dtype=torch.uint8, device=codec.device)
    b = torch.empty_like(a)
    a.fill_(1)
    s = torch.cuda.current_stream(codec.device)
    best = 0.0
    sweep = {}
    names = {0: "x4", 1: "x8", 2: "x16"}
    # forms 16+: LDS-DMA staging (global_load_lds_dwordx4) of 2 / 4 / 8 KiB per wave
    for form in (0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14, 16, 17, 18, 20, 21, 22):
      for g in (1024, 2048, 4096, 8192, 16384, 32768):
        blocks = (form << 24) | g

        def run():
            st = codec.lib.cpk_debug_copy(C.c_void_p(b.data_ptr()), C.c_void_p(a.data_ptr()),
                                          nbytes, blocks, C.c_void_p(s.cuda_stream))
            if st:
                raise RuntimeError(f"cpk_debug_copy: {st}")
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            run()
        e1.record(s)
        torch.cuda.synchronize()
        gbps = 2 * nbytes / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9
        tag = (("lds%dk" % (2 << (form & 3))) if form & 16 else names[form & 3]) + \
            ("nt" if form & 4 else "") + ("c" if form & 8 else "")
        sweep[f"{tag}/{g}"] = round(gbps, 1)
        best = max(best, gbps)
    ok = torch.equal(a, b)
    # the runtime's own device-to-device copy (hipMemcpyAsync: ROCclr's blit kernel), for scale
    b.zero_()
    with torch.cuda.stream(s):
        b.copy_(a)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            b.copy_(a)
        e1.record(s)
        torch.cuda.synchronize()
    sweep["runtime_d2d_copy"] = round(2 * nbytes / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9, 1)
    ok = ok and torch.equal(a, b)
    del a, b
    torch.cuda.empty_cache()
    if not ok:
        raise RuntimeError("copy probe produced wrong bytes")
    return best, sweep


def sha_dev(t, chunk=1 << 28):
    import torch

    b = t.view(torch.uint8) if t.dtype != torch.uint8 else t
    h = hashlib.sha256()
    for i in range(0, b.numel(), chunk):
        h.update(memoryview(b[i : i + chunk].cpu().numpy()))
    return h.hexdigest()


def manifest_entry(name, cfg, seed, first, stride, n):
    p = os.path.join(ROOT, "tests", "golden", "manifest.json")
    if not os.path.exists(p):
        return None
    if cfg.get("stretches"):  # reshaped input: no manifest describes it
        return None
    man = json.load(open(p)).get("configs", {})
    for c in man.values():
        if (c["seed"], c["first_msg"], c["msg_stride"], c["nmsgs"], c["profile"], c["nseg"],
                c["seg_words"]) == (seed, first, stride, n, cfg["profile"], cfg["nseg"],
                                    cfg["seg_words"]):
            return c
    return None


def run_config(name, args, steps, warmup, rank, world, dist, codec):
    import torch

    from capnproto_amd.shard import balanced_ranges, reduce_step, shard_messages

    cfg = CONFIGS[name]

    def barrier():
        if dist is not None:
            dist.barrier()

    mode = args.shard or cfg.get("shard", "block")
    n_global = cfg["nmsgs"] * world
    vrank, vworld = rank, world
    if world == 1 and cfg.get("one_gpu_shard_of"):
        # a config quoted across 8 GPUs, measured on one: its rank-0 shard (the same messages,
        # and the same manifest, as rank 0 of the 8-GPU run)
        vworld = cfg["one_gpu_shard_of"]
        n_global = cfg["nmsgs"] * vworld
    if mode == "bytes":
        goff, _ = codec.gen_offsets(n_global, nseg=cfg["nseg"], seg_words=cfg["seg_words"],
                                    seed=args.seed)
        first, n = balanced_ranges(goff, world)[rank]
        stride = 1
        del goff
    else:
        first, stride, n = shard_messages(vrank, vworld, n_global, mode)
    off, total = codec.gen_offsets(n, nseg=cfg["nseg"], seg_words=cfg["seg_words"],
                                   seed=args.seed, first_msg=first, msg_stride=stride)
    words = codec.gen_messages(cfg["profile"], off, total, nseg=cfg["nseg"], seed=args.seed,
                               first_msg=first, msg_stride=stride)
    if cfg.get("stretches") == "geometric":
        from capnproto_amd.workloads import geometric_stretches

        geometric_stretches(words, off, cfg["nseg"], seed=args.seed, first_msg=first,
                            msg_stride=stride)
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

    # The timed step is one HIP graph (pack + unpack, every launch and scratch memset of the
    # step), captured once and replayed: the same kernels on the same buffers, minus the host's
    # per-launch submission gaps.  --no-graph times the eager launches instead.
    run = step
    graph = None
    if not args.no_graph:
        step()  # every lazily sized scratch buffer and launch setting exists before capture
        codec.sync()
        try:
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                step()
            run = graph.replay
        except Exception as e:  # noqa: BLE001 -- fall back to eager launches, say so
            print(f"bench: graph capture failed ({e}); timing eager launches", file=sys.stderr)
            graph = None
            run = step
    for _ in range(warmup):
        run()
    codec.sync()
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    codec.sync()
    dt = t1 - t0

    # correctness of what was timed: exact round trip + statuses, then the reference's hashes
    checks = {"pack_status": bool((pst == 0).all().item()),
              "unpack_status": bool((ust == 0).all().item()),
              "word_offsets": torch.equal(woff, off),
              "words": torch.equal(back[:total], words[:total])}
    ok = all(checks.values())
    if not ok:
        print(f"bench: {name}: round trip check failed: {checks}", file=sys.stderr)
    man = None if args.no_verify else manifest_entry(name, cfg, args.seed, first, stride, n)
    ref_ok = None
    if man is not None:
        ref_ok = (man["packed_bytes"] == P and sha_dev(packed[:P]) == man["sha256_packed"]
                  and sha_dev(moff) == man["sha256_out_off"])
        if not ref_ok:
            print(f"bench: {name}: packed bytes differ from the reference manifest", file=sys.stderr)
        ok = ok and ref_ok

    # per-kernel durations: a second pass of the same steps with HIP events around every tile
    # kernel, on the stream the kernels run on (kept out of the wall-clock pass above)
    codec.timing_read_all()  # discard
    codec.timing(True)
    for _ in range(steps):
        step()
    codec.timing(False)
    codec.sync()
    kt = codec.timing_read_all()
    kms = {k: (v[0] / v[1] if v[1] else 0.0) for k, v in kt.items()}

    red = reduce_step(dt, float(U), float(P), kms["pack"], kms["unpack"], ok,
                      dist=dist, device=codec.device)
    res = {"name": name, "cfg": cfg, "n": n, "U": U, "P": P, "first": first, "stride": stride,
           "mode": mode, "dt_max": red["dt_max"], "U_all": red["unpacked_all"],
           "ok_all": red["ok_all"], "ref_checked": man is not None, "ref_ok": ref_ok,
           "kms": kms, "steps": steps, "warmup": warmup, "graph": graph is not None}
    res["tensors"] = (words, off, packed, moff, total, cap)
    res["shard"] = (first, stride)
    return res


def summarize(res, world, copy_gbps):
    """Per-config JSON: value, roofline (headline = round trip), dominant kernel."""
    U, P, steps = res["U"], res["P"], res["steps"]
    kms = res["kms"]
    t_step = res["dt_max"] / steps  # seconds, max over ranks
    value = res["U_all"] / t_step / 2**30
    # per-GPU algorithmic bytes of one round trip: pack (read U, write P) + unpack (read P,
    # write U); SURVEY.md 8(d)
    rt = 2.0 * (U + P) / t_step / 1e9
    rd = (U + P) / t_step / 1e9
    algo = {"pack": U + P, "unpack_tiles": U + P}
    kern = {k: {"ms": round(kms[k], 4),
                "GBps": round(algo[k] / (kms[k] * 1e-3) / 1e9, 1) if kms[k] > 0 else None,
                "algorithmic_bytes": int(algo[k])} for k in algo}
    dom = max(algo, key=lambda k: kms[k])
    dom_ach = algo[dom] / (kms[dom] * 1e-3) / 1e9 if kms[dom] > 0 else 0.0
    traffic = None
    tf = os.path.join(ROOT, "profiles", f"traffic_{res['name']}.json")
    if os.path.exists(tf):
        try:
            t = json.load(open(tf))
            if t.get("kernel_src_sha256") == kernel_source_hash():
                traffic = {k: v for k, v in t.items() if k != "kernel_src_sha256"}
        except Exception:
            traffic = None
    cfg = res["cfg"]
    return {
        "value": round(value, 3),
        "ms_per_step": round(t_step * 1e3, 4),
        "config": {
            "workload": cfg["workload"],
            "messages_per_gpu": res["n"],
            "unpacked_bytes_per_gpu": U,
            "packed_bytes_per_gpu": P,
            "packed_ratio": round(P / U, 4),
            "profile": cfg["profile"],
            "shard": res["mode"],
            "parallelism": f"dp{world} (independent message shards, no data-path collective)",
            "launch": "hip graph (one per step)" if res.get("graph") else "eager",
        },
        "parity": ("bit-exact round trip; packed bytes SHA-256 == reference "
                   "(tests/golden/manifest.json)" if res["ref_checked"] else
                   "bit-exact round trip (no reference manifest for this shard)"),
        "roofline": {
            "bound": "hbm",
            "what": "round trip: 2(U+P) algorithmic bytes per GPU per step / wall time of a step",
            "achieved": round(rt, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(rt / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "read_only_frac": round(rd / HBM_PEAK_GBS, 4),
            "measured_copy_GBps": round(copy_gbps, 1) if copy_gbps else None,
            "measured_copy_kernel": "copy_kernel / copy_lds_kernel (cpk_stream.hip): 16 B/lane "
                                    "streaming copy, best of a sweep over loads in flight per "
                                    "lane (4, 8, 16), default or non-temporal access, grid-strided "
                                    "or contiguous blocks, LDS-DMA staging (2 / 4 / 8 KiB per "
                                    "wave), and grid size; read + write bytes, 2 GiB each way",
            "frac_of_measured_copy": round(rt / copy_gbps, 4) if copy_gbps else None,
            "dominant_kernel": {
                "kernel": dom,
                "achieved": round(dom_ach, 1),
                "frac": round(dom_ach / HBM_PEAK_GBS, 4),
                "algorithmic_bytes_per_launch": int(algo[dom]),
            },
            "kernels": kern,
            "pack_ms": round(kms["pack"], 4),
            "unpack_ms": round(kms["unpack"], 4),
        },
    }


def main():
    args = parse()
    bad = [e for e in DEBUG_ENV if os.environ.get(e, "0") not in ("", "0")]
    if bad:
        print(json.dumps({"error": f"diagnostic knob(s) set: {bad}; refusing to report a value"}))
        sys.exit(2)
    knobs = {k: v for k, v in sorted(os.environ.items()) if k.startswith("CPK_")}
    sel = [k for k in KERNEL_ENV if k in knobs]
    if sel and not args.ab:
        print(json.dumps({"error": f"kernel-selection knob(s) set: {sel}; pass --ab for an A/B "
                                   "run (the headline comes from the default kernels)"}))
        sys.exit(2)
    import numpy as np
    import torch

    import capnproto_amd

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

    codec = capnproto_amd.Codec(local)
    copy_gbps, copy_sweep = measure_copy(codec)
    head = run_config(args.config, args, args.steps, args.warmup, rank, world, dist, codec)
    ok = head["ok_all"]
    exchange = None
    if world > 1:
        try:
            exchange = batch_exchange(codec, head, args, rank, world, dist)
        except Exception as e:  # noqa: BLE001 -- reported, never fatal to the timed result
            exchange = {"error": f"{type(e).__name__}: {e}"}

    cb = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb, same = config_cpu_baseline(head, args.cpu_seconds)
        ok = ok and same
    hi = None
    if world == 1 and not args.no_host:
        # the path starts and ends in host memory: serial and pipelined host-inclusive rates
        words, off, packed, moff, total, cap = head["tensors"]
        # two streams, 16 chunks: the best of tools/pcie_probe.py's sweep (the box's PCIe moves
        # about 57 GB/s one way and not much more both ways at once: profiles/r03_pcie_probe.txt)
        extra = [capnproto_amd.Codec(local)]
        hi = {"pipelined": host_inclusive_pipelined([codec] + extra, words, off, total,
                                                    head["n"], moff, min(args.steps, 10),
                                                    chunks=16)}
        for c in extra:
            c.close()
        if args.host_inclusive:
            hi["serial"] = host_inclusive(codec, words, off, total, head["n"], cap, args.steps)
    head.pop("tensors")
    torch.cuda.empty_cache()

    subs = []
    sub = args.sub if args.sub is not None else ("c3,c4,c4g,c5" if world == 1 else "none")
    for nm in [s for s in sub.split(",") if s and s != "none" and s != args.config]:
        r = run_config(nm, args, args.sub_steps, 2, rank, world, dist, codec)
        r["cpu_baseline"] = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            # the reference codec on a bounded sample of this config too (per config)
            r["cpu_baseline"], same = config_cpu_baseline(r, args.cpu_seconds / 2)
            ok = ok and same
        r.pop("tensors")
        torch.cuda.empty_cache()
        ok = ok and r["ok_all"]
        subs.append(r)

    if rank == 0:
        if not ok:
            print(json.dumps({"metric": METRIC, "error": "parity MISMATCH: no value reported",
                              "config": args.config}))
            sys.exit(1)
        s = summarize(head, world, copy_gbps)
        result = {
            "metric": METRIC,
            "value": s["value"],
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": s["ms_per_step"],
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": ("synthetic (deterministic on-device generator, SURVEY.md 8(d))"
                     if not CONFIGS[args.config].get("stretches") else
                     "synthetic (on-device generator, segment bodies rewritten with geometric "
                     "zero stretches by capnproto_amd/workloads.py, seeded per message)"),
            "config": s["config"],
            "parity": s["parity"] + ("; CPU codec packed bytes == device on its sample"
                                     if cb else ""),
            "roofline": s["roofline"],
            "cpu_baseline": cb,
            "kernels": {"pack": "framing + pack_tile (tiles whose offset is known in time write "
                                "straight out; sparse tiles take an exact-size piece of a byte "
                                "arena, dense ones wait for their offset) + pack_place (group "
                                "scan of the tile byte counts, arena copies, requested positions) "
                                "(capnproto_amd/csrc/cpk_pack.hip)",
                        "unpack": "header (+ word-offset scan, tile_first, scratch zeroing) + "
                                  "unpack_tiles (capnproto_amd/csrc/cpk_unpack.hip)",
                        "knobs": knobs},
        }
        result["roofline"]["measured_copy_sweep_GBps"] = {str(k): v for k, v in copy_sweep.items()}
        if subs:
            result["sub_results"] = []
            for r in subs:
                sr = summarize(r, world, copy_gbps)
                sr["steps"] = r["steps"]
                if r.get("cpu_baseline"):
                    sr["cpu_baseline"] = r["cpu_baseline"]
                result["sub_results"].append(sr)
        if hi is not None:
            result["host_inclusive"] = hi
        if exchange is not None:
            result["batch_exchange"] = exchange
        if not args.no_host:
            result["small_message_latency"] = small_message_latency(codec)
        if not args.no_split and world == 1:
            result["stream_split"] = split_bench(codec, args.seed)
        print(json.dumps(result))
    codec.close()
    if dist is not None:
        dist.destroy_process_group()


def batch_exchange(codec, head, args, rank, world, dist, reps=3):
    """The batch case at N > 1: every rank's packed bytes gathered onto rank 0
    at their global offsets (capnproto_amd.shard.gather_packed: an all-gather of per-rank totals,
    then RCCL send/recv over xGMI into slices of rank 0's buffer), outside the timed step.
    Timed on every rank between barriers; rank 0 then unpacks the gathered stream with the
    global offsets and checks it against the global batch regenerated on the device (round-robin
    shards included: gather_packed places every message at its global index).  Reported as its own number, never folded into `value`."""
    import torch

    from capnproto_amd.shard import gather_packed

    words, off, packed, moff, total, cap = head["tensors"]
    first, stride = head["shard"]
    n = head["n"]
    times = []
    out = offs = None
    for _ in range(reps):
        out = offs = None
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        out, offs = gather_packed(packed, moff, n, dst=0, dist=dist, device=codec.device,
                                  first_msg=first, msg_stride=stride, codec=codec)
        torch.cuda.synchronize()
        dist.barrier()
        times.append(time.perf_counter() - t0)
    t = min(times)
    if rank != 0:
        return None
    G = int(offs[-1].item())
    res = {"to_rank": 0, "ranks": world, "packed_bytes": G, "ms": round(1e3 * t, 3),
           "GBps": round(G / t / 1e9, 2),
           "what": "all ranks' packed bytes + message offsets gathered onto rank 0 at their "
                   "global offsets (all-gather of totals, then RCCL send/recv)"}
    cfg = CONFIGS[args.config]
    nglob = int(offs.numel()) - 1
    if G > (24 << 30):
        res["verified"] = "skipped (gathered stream too large to re-decode beside the batch)"
        return res
    U = head["U_all"]
    back, woff, ust = codec.unpack_messages(out, offs, int(U) // 8, nbytes=G)
    codec.sync()
    ok = bool((ust == 0).all().item()) and int(woff[-1].item()) * 8 == int(U)
    if ok:  # (message k of the global batch at position k, whatever the shard assignment)
        goff, gtot = codec.gen_offsets(nglob, nseg=cfg["nseg"], seg_words=cfg["seg_words"],
                                       seed=args.seed)
        gw = codec.gen_messages(cfg["profile"], goff, gtot, nseg=cfg["nseg"], seed=args.seed)
        if cfg.get("stretches") == "geometric":
            from capnproto_amd.workloads import geometric_stretches

            geometric_stretches(gw, goff, cfg["nseg"], seed=args.seed)
        ok = torch.equal(woff, goff) and torch.equal(back[:gtot], gw[:gtot])
        del gw, goff
    res["round_trip_exact"] = ok
    del back, out
    torch.cuda.empty_cache()
    return res


def split_bench(codec, seed, n=1 << 20, reps=5):
    """Stream boundary discovery (cpk_split_packed_stream) on a C5-shaped
    stream: 1 Mi messages of 2^k + 1 words (k in 3..11), mixed profiles, packed back to back with
    no index.  Timed: the whole split (flat decode of the stream + the block-parallel walk over
    the message headers), device-resident; checked against the generator's layout."""
    torch = codec.torch
    off, total = codec.gen_offsets(n, seed=seed + 5)
    words = codec.gen_messages("mixed", off, total, seed=seed + 5)
    packed, poff, st = codec.pack_messages(words, off)
    codec.sync()
    nbytes = int(poff[-1].item())
    out = torch.empty(total + 16, dtype=torch.int64, device=codec.device)
    res = None
    times = []
    for i in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = codec.split_packed_stream(packed, total + 16, n + 1, nbytes=nbytes, words=out)
        codec.sync()
        if i:
            times.append(time.perf_counter() - t0)
    w2, woff, ioff, status, cnt = res
    ok = (int(cnt.item()) == n and int(status[n].item()) == 0 and torch.equal(woff[:n + 1], off)
          and torch.equal(ioff[:n + 1], poff) and torch.equal(w2[:total], words[:total]))
    t = min(times)
    del words, packed, out, w2
    return {"messages": n, "unpacked_bytes": 8 * total, "packed_bytes": nbytes,
            "ms": round(1e3 * t, 3), "GiBps": round(8 * total / t / 2**30, 2),
            "split_exact": bool(ok),
            "what": "flat decode of the stream + block-parallel message-chain walk; unpacked "
                    "GiB/s, device-resident, wall clock of the call incl. its sync"}


def small_message_latency(codec, reps=300):
    """Per-call latency of the host entry points on one small message -- the addressbook sample
    (tests/golden/addressbook.bin, 288 B: the reference's samples/addressbook.c++ message), as
    writePackedMessage / PackedMessageReader over the C++ facade would call them: pinned-less
    host buffers, upload, the kernels, a sync, download."""
    import ctypes as C
    import numpy as np
    src = os.path.join(ROOT, "tests", "golden", "addressbook.bin")
    words = np.frombuffer(open(src, "rb").read(), "<u8").copy()
    n = len(words)
    off = np.array([0, n], "<u8")
    cap = 8 * n + n + 16
    out = np.zeros(cap, np.uint8)
    oo = np.zeros(2, "<u8")
    st = np.zeros(1, "<i4")
    back = np.zeros(n, "<u8")
    wo = np.zeros(2, "<u8")
    lib = codec.lib
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    t_pack, t_unpack = [], []
    for i in range(reps + 20):
        t0 = time.perf_counter()
        r1 = lib.cpk_pack_messages_host(codec.ctx, p(words), n, p(off), 1, p(out), cap, p(oo), p(st))
        t1 = time.perf_counter()
        P = int(oo[1])
        r2 = lib.cpk_unpack_messages_host(codec.ctx, p(out), P, p(oo), 1, p(back), n, p(wo), p(st),
                                          None)
        t2 = time.perf_counter()
        if r1 or r2:
            return {"error": [int(r1), int(r2)]}
        if i >= 20:
            t_pack.append(t1 - t0)
            t_unpack.append(t2 - t1)
    ok = bool((back == words).all())
    return {"message_bytes": 8 * n, "packed_bytes": P, "round_trip_exact": ok,
            "pack_us_median": round(1e6 * float(np.median(t_pack)), 1),
            "unpack_us_median": round(1e6 * float(np.median(t_unpack)), 1),
            "calls": reps,
            "path": "cpk_pack_messages_host / cpk_unpack_messages_host (H2D, kernels, sync, D2H) "
                    "on the addressbook sample"}


def host_inclusive_pipelined(codecs, words, off, total, n, moff, steps, chunks=8):
    """The same host-to-host path, chunked by messages and pipelined over S streams, each with
    its own codec context: chunk i runs H2D(U_i) -> pack -> D2H(P_i) -> H2D(P_i) -> unpack ->
    D2H(U_i) in order on stream i % S, so one stream's uploads overlap another's downloads and
    both PCIe directions run at once (no cross-stream waits: a wait on another stream's event
    stalls the hardware queue both streams may share; tools/host_sweep.py measures S and the
    chunk count).  The packed size of each chunk is what
    the caller's framing knows (moff, learned once before timing, as the serial path does)."""
    import torch

    dev = codecs[0].device
    offh = off.cpu()
    mo = moff.cpu()
    per = (n + chunks - 1) // chunks
    cuts = [(i * per, min(n, (i + 1) * per)) for i in range(chunks) if i * per < n]
    hw = torch.empty(total, dtype=torch.int64, pin_memory=True)
    hw.copy_(words[:total])
    P = int(mo[-1])
    hp = torch.empty(P, dtype=torch.uint8, pin_memory=True)
    hb = torch.empty(total, dtype=torch.int64, pin_memory=True)
    dw = torch.empty(total, dtype=torch.int64, device=dev)
    dp = torch.empty(P + 64, dtype=torch.uint8, device=dev)
    dp2 = torch.empty(P + 64, dtype=torch.uint8, device=dev)
    back = torch.empty(total, dtype=torch.int64, device=dev)
    streams = [torch.cuda.Stream(dev) for _ in codecs]
    parts = []
    for i, (a, b) in enumerate(cuts):
        w0, w1 = int(offh[a]), int(offh[b])
        p0, p1 = int(mo[a]), int(mo[b])
        parts.append(dict(w0=w0, w1=w1, p0=p0, p1=p1, k=i % len(codecs),
                          off=(off[a:b + 1] - w0).contiguous(),
                          poff=(moff[a:b + 1] - p0).contiguous(),
                          moff=torch.empty(b - a + 1, dtype=torch.int64, device=dev),
                          woff=torch.empty(b - a + 1, dtype=torch.int64, device=dev),
                          st=torch.empty(max(b - a, 1), dtype=torch.int32, device=dev),
                          ust=torch.empty(max(b - a, 1), dtype=torch.int32, device=dev)))

    def step():
        for q in parts:
            w0, w1, p0, p1 = q["w0"], q["w1"], q["p0"], q["p1"]
            s, c = streams[q["k"]], codecs[q["k"]]
            with torch.cuda.stream(s):
                dw[w0:w1].copy_(hw[w0:w1], non_blocking=True)
                c.pack_messages(dw[w0:w1], q["off"], out=dp[p0:], msg_out_off=q["moff"],
                                status=q["st"], stream=s)
                hp[p0:p1].copy_(dp[p0:p1], non_blocking=True)
                dp2[p0:p1].copy_(hp[p0:p1], non_blocking=True)
                c.unpack_messages(dp2[p0:], q["poff"], w1 - w0, nbytes=p1 - p0, words=back[w0:],
                                  msg_word_off=q["woff"], status=q["ust"], stream=s)
                hb[w0:w1].copy_(back[w0:w1], non_blocking=True)

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    ok = torch.equal(hb, hw) and bytes(hp.numpy()) == bytes(dp[:P].cpu().numpy())
    return {"GiBps": round(total * 8 / dt / 2**30, 3), "ms_per_step": round(dt * 1e3, 3),
            "round_trip_exact": bool(ok), "chunks": len(cuts), "streams": len(codecs),
            "path": "pinned H2D(U) + pack + D2H(P) + H2D(P) + unpack + D2H(U), chunked by "
                    "messages over several streams / contexts (one stream's uploads overlap "
                    "another's downloads)"}


def host_inclusive(codec, words, off, total, n, cap, steps):
    """U / (H2D(U) + pack + D2H(P) + H2D(P) + unpack + D2H(U)) with pinned host buffers: the
    path starting and ending in host memory.  Serial: one stream, every copy waits for the
    previous stage."""
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
    ok = torch.equal(hb, hw)
    return {"GiBps": round(total * 8 / dt / 2**30, 3), "ms_per_step": round(dt * 1e3, 3),
            "round_trip_exact": bool(ok),
            "path": "pinned H2D(U) + pack + D2H(P) + H2D(P) + unpack + D2H(U), one stream"}


if __name__ == "__main__":
    main()
