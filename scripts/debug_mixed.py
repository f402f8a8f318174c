"""Debug helper (not a test): decode the config-4 mixed batch on the GPU and
report every run whose boundary did not match (entry vs the true frame starts
from the generator's table).

usage: python scripts/debug_mixed.py [extra opts hex]
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from xynet_amd import _lib  # noqa: E402
from xynet_amd import websocket as ws  # noqa: E402

xo = int(sys.argv[1], 0) if len(sys.argv) > 1 else 0
T = _lib.load_tools()
buf, info = bench.build_batch(torch, T, "c4", 0, 1)
tot = C.c_uint64()
n = T.xyws_tools_mixed_table(info["seed"], 1 << 30, None, 0, C.byref(tot))
tab = torch.empty(n * 32, dtype=torch.uint8)
T.xyws_tools_mixed_table(info["seed"], 1 << 30, C.c_void_p(tab.data_ptr()), n, C.byref(tot))
rec = np.frombuffer(tab.numpy().tobytes(), dtype=np.dtype(
    [("off", "<u8"), ("plen", "<u8"), ("draw", "<u8"), ("b0", "u1"), ("hlen", "u1"), ("pad", "u1", 6)]))
starts = rec["off"].astype(np.int64)
sset = set(starts.tolist())
dec = ws.frame_decoder()
dec.opts |= xo
# the bench decodes the same buffer repeatedly (payloads alternate masked /
# unmasked); find the first decode with a bad boundary
NONE = (1 << 64) - 1
for it in range(int(os.environ.get("ITERS", "12"))):
    dec.opts |= 0x100
    dec.decode(buf, cap=0, count=False, carry=False)
    torch.cuda.synchronize()
    st = (C.c_uint64 * 32)()
    dec.ctx.L.xyws_debug_stats(dec.ctx.h, st)
    print("decode", it, "bad", st[2], "repairs", st[3])
    if st[2]:
        break
out = (C.c_uint64 * 32)()
dec.ctx.L.xyws_debug_stats(dec.ctx.h, out)
print("stats", list(out)[:16])
R = (C.c_uint64 * (24 * 1024))()
nr = dec.ctx.L.xyws_debug_records(dec.ctx.h, R, 1024)
r = np.frombuffer(R, dtype=np.uint64).reshape(-1, 24)[:nr]
NONE = (1 << 64) - 1
for i in range(nr):
    h, W, ok = int(r[i, 0]), int(r[i, 1]), int(r[i, 8])
    if h == NONE and W == NONE and ok == 0 and i > 0:
        continue
    okb, succ = ok & 1, ok >> 32
    bad_entry = h != NONE and h not in sset
    if not okb or bad_entry:
        hn, first = int(r[i, 9]), int(r[i, 13])
        j = int(np.searchsorted(starts, h, side="right")) - 1 if h != NONE else -1
        print(f"run {i}: h={h} W={W} entry_true={h in sset} ok={okb} succ={succ} hn={hn} "
              f"hn_true={hn in sset} first_after={first} first_true={first in sset} "
              f"frame_before_h: off={starts[j] if j >= 0 else None} plen={rec['plen'][j] if j >= 0 else None}")
buf2, _ = bench.build_batch(torch, T, "c4", 0, 1)
if it % 2 == 1:  # the decode that failed saw the payloads unmasked once more
    dec2 = ws.frame_decoder()
    for _ in range(it):
        dec2.decode(buf2, cap=0, count=False, carry=False)
    torch.cuda.synchronize()
for i in range(nr):
    h = int(r[i, 0])
    if h != (1 << 64) - 1 and h not in sset:
        b = buf2[h - 16:h + 48].cpu().numpy()
        print(f"run {i} bytes around h (h at +16):", " ".join(f"{x:02x}" for x in b))
        rb = i * (int(info["size"]) + 255) // 256
        print("  range start approx", i * ((info["size"] + 255) // 256 + 15 & ~15))
