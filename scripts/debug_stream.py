"""Debug helper (not a test): decode a named golden stream on the GPU and
report where the output differs from the oracle, plus decoder stats.

usage: python scripts/debug_stream.py [case] [mode: fused|runs1k|serial]
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import streams  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402
from xynet_amd import websocket as ws  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "random_frames_40"
mode = sys.argv[2] if len(sys.argv) > 2 else "fused"
split = int(sys.argv[3]) if len(sys.argv) > 3 else 0
kw = {"fused": {}, "runs1k": {"small_segments": True}, "serial": {"serial": True}}[mode]
src = streams.case_bytes(name)
orc = Oracle()
ob = np.frombuffer(src, np.uint8).copy()
ofr, oc, on = orc.decode_stream(ob)
t = torch.frombuffer(bytearray(src), dtype=torch.uint8).cuda()
dec = ws.frame_decoder(**kw)
dec.opts |= 0x100
if split:
    a = t[:split].clone()
    b = t[split:].clone()
    ra = dec.decode(a, cap=on + 4)
    print("carry after piece 1:", list(bytes(dec.carry())[:40]))
    r = dec.decode(b, cap=on + 4)
    t = torch.cat([a, b])
else:
    r = dec.decode(t, cap=on + 4)
out = (C.c_uint64 * 32)()
dec.ctx.L.xyws_debug_stats(dec.ctx.h, out)
print("len", len(src), "nframes gpu", r.nframes, "oracle", on)
print("stats", list(out)[:8], "err", dec.ctx.last_device_error())
got = t.cpu().numpy()
diff = np.nonzero(got != ob)[0]
print("differing bytes:", diff.size)
if diff.size:
    starts = [f.frame_off for f in ofr]
    runs = []
    a = diff[0]
    prev = a
    for d in diff[1:]:
        if d != prev + 1:
            runs.append((a, prev + 1))
            a = d
        prev = d
    runs.append((a, prev + 1))
    for a, b in runs[:20]:
        i = int(np.searchsorted(starts, a, side="right")) - 1
        f = ofr[i] if i >= 0 else None
        print(f"  diff [{a}, {b}) len {b - a} seg {a // 131072} off-in-seg {a % 131072}; "
              f"frame#{i} start {f.frame_off if f else None} ps {f.payload_off if f else None} "
              f"plen {f.payload_len if f else None}")
gfr = r.frames()
for i, (g, o) in enumerate(zip(gfr, ofr)):
    if (g.frame_off, g.payload_len) != (o.frame_off, o.payload_len):
        print("first frame mismatch at", i, (g.frame_off, g.payload_len), (o.frame_off, o.payload_len))
        break
