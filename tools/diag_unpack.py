"""Unpack step counters from a diagnostic build (tools/build_variant.sh diag -DCPK_DIAG).

    python3 tools/diag_unpack.py capnproto_amd/var_diag.so c2 c3 c4

Packs and unpacks each bench config once (untimed), then prints the per-tile averages of the
counters cpk_debug_diag documents (cpk_unpack.hip).
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import capnproto_amd  # noqa: E402

capnproto_amd.LIB_PATH = os.path.abspath(sys.argv[1])
import torch  # noqa: E402

from bench import CONFIGS  # noqa: E402

NAMES = ["tiles", "walk0_trips", "walk0_lane_steps", "rewalk_trips", "rewalk_lane_steps",
         "settle_rounds", "enter_calls", "merge_steps", "merge_capped", "entry_mismatch",
         "opt_walked", "has_start", "f_cand", "f_used", "not_ok", "lb_first_read_ticks",
         "clk_stage", "clk_chain0", "clk_wait_x0p", "clk_entry", "clk_lookback", "clk_expand",
         "lb_windows", "lb_wait_unpub", "lb_wait_incl", "lb_polls", "incl_waits", "unpublished",
         "win_before_wait", "win_resolved"]

L = capnproto_amd.load_library()
L.cpk_debug_diag.restype = C.c_int
L.cpk_debug_diag.argtypes = [C.c_void_p, C.c_int]
L.cpk_debug_pdiag.restype = C.c_int
L.cpk_debug_pdiag.argtypes = [C.c_void_p, C.c_int]
pbuf = (C.c_uint64 * 4)()
TL_N = 1 << 16
tl = None
if hasattr(L, "cpk_debug_timeline"):
    L.cpk_debug_timeline.restype = C.c_int
    L.cpk_debug_timeline.argtypes = [C.c_void_p, C.c_int]
    tl = (C.c_uint64 * (8 * TL_N))()


ptl = None
if hasattr(L, "cpk_debug_ptimeline"):
    L.cpk_debug_ptimeline.restype = C.c_int
    L.cpk_debug_ptimeline.argtypes = [C.c_void_p, C.c_int]
    ptl = (C.c_uint64 * (8 * TL_N))()


def ptimeline(name):
    """Per-tile wall-clock phases of the first pack tiles of the last pack_tile launch."""
    if ptl is None:
        return
    assert L.cpk_debug_ptimeline(ptl, TL_N) == 0
    import numpy as np
    a = np.frombuffer(ptl, dtype=np.uint64).reshape(TL_N, 8).astype(np.int64)
    a = a[a[:, 0] > 0]
    if len(a) == 0:
        return
    t0 = a[:, 0].min()
    w = (a[:, :5] - t0) / 100.0
    pct = lambda v: " ".join(f"{q}:{np.percentile(v, q):.2f}" for q in (10, 50, 90, 99))
    print(f"{name} pack timeline tiles {len(a)} span_us {w[:, 4].max():.1f} start_us [{pct(w[:, 0])}]"
          f" life_us [{pct(w[:, 4] - w[:, 0])}]", flush=True)
    for k, nm in enumerate(["analysis", "emission", "decision", "copy_out"]):
        v = w[:, k + 1] - w[:, k]
        print(f"  {nm:9s} mean {v.mean():7.3f} us  [{pct(v)}]", flush=True)
    bw = a[:, 7] / 100.0
    print(f"  budget wait (wave 0) mean {bw.mean():.3f} us [{pct(bw)}] share waiting {np.mean(bw > 0):.3f}", flush=True)
    for o, nm in ((1, "in_time"), (2, "slot"), (3, "waited")):
        sel = a[:, 5] == o
        if sel.any():
            print(f"  {nm:8s} {sel.mean():.3f} decision {np.mean(w[sel, 3] - w[sel, 2]):.2f} us"
                  f" life {np.mean(w[sel, 4] - w[sel, 0]):.2f} us", flush=True)
    hist = np.bincount((w[:, 0] // 5).astype(np.int64))
    print("  starts/5us", " ".join(str(int(x)) for x in hist[:60]), flush=True)
    # the look-back distance: tiles between t and the nearest tile whose decision (offset) was
    # known before t's staging ended
    dec = w[:, 3]
    ready = w[:, 2]
    n = len(a)
    dist = []
    for t in range(1, n, max(1, n // 2000)):
        lo = max(0, t - 8192)
        known = np.nonzero(dec[lo:t] <= ready[t])[0]
        dist.append(t - (lo + known[-1]) if len(known) else 8192)
    print(f"  nearest resolved predecessor at staging end (tiles) [{pct(np.array(dist))}]", flush=True)


def timeline(name, ntiles):
    """Per-tile wall-clock phases (10 ns ticks) of the first tiles of the last unpack launch."""
    if tl is None:
        return
    assert L.cpk_debug_timeline(tl, TL_N) == 0
    import numpy as np
    n = min(ntiles, TL_N)
    a = np.frombuffer(tl, dtype=np.uint64).reshape(TL_N, 8)[:n].astype(np.int64)
    a = a[a[:, 0] > 0]
    if len(a) == 0:
        return
    t0 = a[:, 0].min()
    w = (a[:, :7] - t0) / 100.0  # us from the first tile's start
    ph = np.diff(w, axis=1)
    names = ["stage", "chain0", "wait_x0p", "entry", "lookback", "expand"]
    pct = lambda v: " ".join(f"{q}:{np.percentile(v, q):.2f}" for q in (10, 50, 90, 99))
    print(f"{name} timeline tiles {len(a)} span_us {w[:, 6].max():.1f} start_us [{pct(w[:, 0])}]"
          f" end_us [{pct(w[:, 6])}] life_us [{pct(w[:, 6] - w[:, 0])}]", flush=True)
    for k, nm in enumerate(names):
        print(f"  {nm:9s} mean {ph[:, k].mean():7.3f} us  [{pct(ph[:, k])}]", flush=True)
    # starts per 5 us bucket (dispatch / occupancy), and the look-back wait against the time its
    # predecessor tile finished its own look-back (t - 1's wk5) when that came later
    hist = np.bincount((w[:, 0] // 5).astype(np.int64))
    print("  starts/5us", " ".join(str(int(x)) for x in hist[:60]), flush=True)
    hw = a[:, 7]
    cu = (hw >> 8) & 0xF
    se = (hw >> 13) & 0x7
    xcd = np.arange(len(a)) // 4 % 8
    for x in range(8):
        sel = xcd == x
        if sel.any():
            print(f"  xcd{x} life {np.mean(w[sel, 6] - w[sel, 0]):.2f} chain0 {ph[sel, 1].mean():.2f}"
                  f" wait {ph[sel, 2].mean():.2f} lookback {ph[sel, 4].mean():.2f}"
                  f" expand {ph[sel, 5].mean():.2f}", flush=True)
    # resolution (end of the look-back) per 10 us, and how far behind its own readiness a tile
    # resolves compared with the tile before it
    res = np.bincount((w[:, 5] // 10).astype(np.int64))
    print("  resolved/10us", " ".join(str(int(x)) for x in res[:80]), flush=True)
    lagp = w[1:, 5] - w[:-1, 5]
    print(f"  resolve t minus t-1 us [{pct(lagp)}]", flush=True)
    gap = w[1:, 2] - w[:-1, 2]  # x0p publish: tile t's minus tile t - 1's
    print(f"  x0p publish t minus t-1 us [{pct(gap)}]  se values {np.unique(se)[:8]} cu {np.unique(cu)[:16]}",
          flush=True)
def flat_entry_detail():
    """Flat decode: where the slow entries go -- AGG publication (wa: ticks after the tile's
    start) and the predecessor's AGG seen (wb), from slot 7 of the diagnostic timeline."""
    if tl is None:
        return
    import numpy as np
    a = np.frombuffer(tl, dtype=np.uint64).reshape(TL_N, 8).astype(np.int64)
    ok = a[:, 0] > 0
    idx = np.nonzero(ok)[0]
    a = a[ok]
    wa = (a[:, 7] & 0xffffffff) / 100.0
    wb = (a[:, 7] >> 32) / 100.0
    ent = (a[:, 4] - a[:, 3]) / 100.0
    pct = lambda v: " ".join(f"{q}:{np.percentile(v, q):.2f}" for q in (10, 50, 90, 99))
    print(f"  flat: AGG published at [{pct(wa)}] us; waited for predecessor's AGG [{pct(wb - wa)}] us;"
          f" after it [{pct((a[:, 4] - a[:, 0]) / 100.0 - wb)}] us", flush=True)
    slow = np.argsort(-ent)[:12]
    t0 = a[:, 0].min()
    for j in slow:
        t = idx[j]
        print(f"   slow entry tile {t} (t%4={t % 4}) entry {ent[j]:.1f} start {(a[j, 0] - t0) / 100:.1f}"
              f" agg@{wa[j]:.1f} pred_agg_seen@{wb[j]:.1f} chain0 {(a[j, 2] - a[j, 1]) / 100:.1f}", flush=True)
    w4 = np.array([ent[(idx % 4) == k].mean() for k in range(4)])
    print("  flat: entry mean by wave", " ".join(f"{x:.2f}" for x in w4), flush=True)


codec = capnproto_amd.Codec(0)
buf = (C.c_uint64 * 32)()
for name in sys.argv[2:]:
    if name == "split":
        # the bench's stream split: the whole stream decoded as one flat chunk
        n = 1 << 20
        off, total = codec.gen_offsets(n, seed=7)
        words = codec.gen_messages("mixed", off, total, seed=7)
        packed, poff, st = codec.pack_messages(words, off)
        codec.sync()
        nbytes = int(poff[-1].item())
        codec.split_packed_stream(packed, total + 16, n + 1, nbytes=nbytes)  # (warm)
        codec.sync()
        L.cpk_debug_diag(buf, 1)
        if tl is not None:
            L.cpk_debug_timeline(tl, TL_N)
        res = codec.split_packed_stream(packed, total + 16, n + 1, nbytes=nbytes)
        codec.sync()
        assert L.cpk_debug_diag(buf, 1) == 0
        timeline(name, 1 << 30)
        flat_entry_detail()
        t = max(buf[0], 1)
        print(name, "messages", int(res[4].item()), "tiles", buf[0], " ".join(
            f"{NAMES[k]}={buf[k] / t:.3f}" for k in range(1, len(NAMES)) if NAMES[k] != "-"), flush=True)
        del words, packed, res
        torch.cuda.empty_cache()
        continue
    cfg = CONFIGS[name]
    n = cfg["nmsgs"]
    off, total = codec.gen_offsets(n, nseg=cfg["nseg"], seg_words=cfg["seg_words"], seed=1)
    words = codec.gen_messages(cfg["profile"], off, total, nseg=cfg["nseg"], seed=1)
    cap = codec.packed_bound(total, n * (cfg["nseg"] + 1)) + 64
    packed = torch.empty(cap, dtype=torch.uint8, device=codec.device)
    moff = torch.empty(n + 1, dtype=torch.int64, device=codec.device)
    back = torch.empty(total, dtype=torch.int64, device=codec.device)
    codec.pack_messages(words, off, out=packed, msg_out_off=moff)  # (first call: allocations)
    codec.sync()
    L.cpk_debug_pdiag(pbuf, 1)
    if ptl is not None:
        L.cpk_debug_ptimeline(ptl, TL_N)
    codec.pack_messages(words, off, out=packed, msg_out_off=moff)
    codec.sync()
    assert L.cpk_debug_pdiag(pbuf, 1) == 0
    print(name, "pack tiles", pbuf[0], "in_time", pbuf[1], "slot", pbuf[2], "waited", pbuf[3], flush=True)
    ptimeline(name)
    P = int(moff[-1].item())
    codec.unpack_messages(packed, moff, total, nbytes=P, words=back)  # (warm: allocations)
    codec.sync()
    L.cpk_debug_diag(buf, 1)
    if tl is not None:
        L.cpk_debug_timeline(tl, TL_N)
    codec.unpack_messages(packed, moff, total, nbytes=P, words=back)
    codec.sync()
    assert L.cpk_debug_diag(buf, 1) == 0
    timeline(name, 1 << 30)
    ok = torch.equal(back[:total], words[:total])
    t = max(buf[0], 1)
    print(name, "round_trip", ok, "tiles", buf[0], " ".join(
        f"{NAMES[k]}={buf[k] / t:.3f}" for k in range(1, len(NAMES)) if NAMES[k] != "-"), flush=True)
    del words, packed, back, moff, off
    torch.cuda.empty_cache()
