"""Phase split of the run decoder on an echo-sized batch: 0-1000 B masked
text frames (the loopback echo harness's traffic), descriptors on, several
calls on one stream (policy words set), then two calls with XYWS_OPT_STATS.
Prints the per-call HIP-event time and the decoder's counters (cycles per run
at 2.1 GHz) as one JSON line.  usage: small_batch_stats.py [BYTES] [OPTS]"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import streams  # noqa: E402
from xynet_amd import _lib, websocket as ws  # noqa: E402

size = int(sys.argv[1], 0) if len(sys.argv) > 1 else 4 << 20
xo = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0
rng = streams.SplitMix(0xEC40)
b = bytearray()
while len(b) < size:
    b += streams.frame(rng, 0x81, rng.next() % 1001)
src = bytes(b[:size])
dev = torch.frombuffer(bytearray(src), dtype=torch.uint8).cuda()
dec = ws.frame_decoder(opts=xo)
cap = size // 6 + 2
for _ in range(5):
    dev.copy_(torch.frombuffer(bytearray(src), dtype=torch.uint8))
    r = dec.decode(dev, cap=cap, carry=False)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20):
    r = dec.decode(dev, cap=cap, carry=False)
e.record()
torch.cuda.synchronize()
us = s.elapsed_time(e) / 20 * 1e3
stream = torch.cuda.current_stream()
names = ["runs", "runs_without_entry", "bad_boundaries", "repairs", "cuts", "spins", "dense_passes",
         "frames", "scan_segments", "scan_survivors", "scan_undecided", "cyc_scan_filter",
         "cyc_scan_check", "cyc_scan_resolve", "cyc_dense_entry", "cyc_dense_chase", "cyc_prologue", "cyc_main",
         "cyc_wait", "cyc_fill", "cyc_chase_sync", "cyc_xor", "cyc_tail", "cyc_prefetch_issue", "cyc_chase_pass",
         "cyc_pro_fill", "cyc_pro_scan", "cyc_pro_publish", "dense_no_entry", "dense_chase_fail",
         "dense_mismatch", "dense_overflow", "giveups", "bridges", "steal_requests", "steals",
         "stolen_segments", "cyc_dense_validate", "cyc_rows", "cyc_serial_chase", "p_lattice", "x41", "x42",
         "x43", "x44", "x45", "cyc_stride_pass"]
out = (C.c_uint64 * _lib.NSTATS)()
for _ in range(2):
    dec.opts = xo | _lib.OPT_STATS
    dec.decode(dev, cap=cap, carry=False)
    dec.ctx.L.xyws_debug_stats(dec.ctx.h, C.c_void_p(stream.cuda_stream), out)
pol = (C.c_uint64 * 5)()
dec.ctx.L.xyws_debug_policy(dec.ctx.h, C.c_void_p(stream.cuda_stream), pol)
st = dict(zip(names, list(out)))
nrun = max(1, st["runs"])
for k in list(st):
    if k.startswith("cyc_"):
        st[k.replace("cyc_", "us_per_run_")] = round(st.pop(k) / nrun / 2100.0, 2)
print(json.dumps({"bytes": size, "opts": xo, "frames": r.nframes, "us_per_call": round(us, 1),
                  "policy": list(pol), "stats": st}))
