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
         "opt_walked", "has_start", "f_cand", "f_used", "not_ok", "-",
         "clk_stage", "clk_chain0", "clk_wait_x0p", "clk_entry", "clk_lookback", "clk_expand"]

L = capnproto_amd.load_library()
L.cpk_debug_diag.restype = C.c_int
L.cpk_debug_diag.argtypes = [C.c_void_p, C.c_int]
L.cpk_debug_pdiag.restype = C.c_int
L.cpk_debug_pdiag.argtypes = [C.c_void_p, C.c_int]
pbuf = (C.c_uint64 * 4)()
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
        L.cpk_debug_diag(buf, 1)
        res = codec.split_packed_stream(packed, total + 16, n + 1, nbytes=nbytes)
        codec.sync()
        assert L.cpk_debug_diag(buf, 1) == 0
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
    codec.pack_messages(words, off, out=packed, msg_out_off=moff)
    codec.sync()
    assert L.cpk_debug_pdiag(pbuf, 1) == 0
    print(name, "pack tiles", pbuf[0], "in_time", pbuf[1], "slot", pbuf[2], "waited", pbuf[3], flush=True)
    P = int(moff[-1].item())
    L.cpk_debug_diag(buf, 1)
    codec.unpack_messages(packed, moff, total, nbytes=P, words=back)
    codec.sync()
    assert L.cpk_debug_diag(buf, 1) == 0
    ok = torch.equal(back[:total], words[:total])
    t = max(buf[0], 1)
    print(name, "round_trip", ok, "tiles", buf[0], " ".join(
        f"{NAMES[k]}={buf[k] / t:.3f}" for k in range(1, len(NAMES)) if NAMES[k] != "-"), flush=True)
    del words, packed, back, moff, off
    torch.cuda.empty_cache()
