import ctypes as C, os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests", "golden")); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np, torch, streams
from xynet_amd import websocket as ws
for fake in (0, 1, 2):
    rng = streams.SplitMix(0xDE5E + fake)
    out = bytearray()
    while len(out) < (3 << 20):
        plen = 120 + rng.below(400)
        key = rng.bytes(4)
        if fake == 0:
            wire = rng.bytes(plen)
        else:
            unit = (bytes([0x82, 0x81]) + rng.bytes(5)) if fake == 1 else (bytes([0x82, 0xFE, 0x00, 0x40]) + rng.bytes(4) + rng.bytes(64))
            off = rng.below(len(unit))
            wire = (rng.bytes(off) + unit * (plen // len(unit) + 2))[:plen]
        out += streams.header(0x82, plen, key, None) + wire
    t = torch.frombuffer(bytearray(out), dtype=torch.uint8).cuda()
    dec = ws.frame_decoder()
    dec.opts |= 0x100
    dec.decode(t, cap=0, count=False, carry=False)
    st = (C.c_uint64 * 32)()
    dec.ctx.L.xyws_debug_stats(dec.ctx.h, st)
    print(fake, "runs", st[0], "dense", st[6], "noent/chase/mism/ovf", list(st)[28:32], "bad", st[2], "rep", st[3])
