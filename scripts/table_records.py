"""Table decoder records of one config batch decoded with XYWS_OPT_TABLE (debug aid):
run entries, exits, frame counts, skips and the per-run index-phase timings.
  usage: table_records.py [CONFIG_NAME]"""
import sys, os, ctypes as C, json
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path.insert(0, os.path.join(ROOT, 'tests')); sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden')); sys.path.insert(0, ROOT)
import numpy as np, torch
from test_gpu_parity import tools_batch, dev_digest
from xynet_amd import websocket as ws
name = sys.argv[1] if len(sys.argv) > 1 else "t_bin_64k_x64"
buf, c = tools_batch(name)
dec = ws.frame_decoder(opts=0x10000000)
r = dec.decode(buf, cap=0)
s = torch.cuda.current_stream()
W = 64 + 3072
out = (C.c_uint64 * (W + 1024 * 16))()
n = dec.ctx.L.xyws_debug_table(dec.ctx.h, C.c_void_p(s.cuda_stream), out, len(out))
w = list(out)
print("n", n, "frames", r.nframes, c["decoded_frames"], "digest ok", dev_digest(buf) == c["out_digest"])
print("ctl", w[:8])
NONE = (1 << 64) - 1
R = w[2] if w[2] else 256
t0 = min(w[W + 16 * i + 5] for i in range(R))
sc = [(w[W + 16 * i + 6] - w[W + 16 * i + 5]) / 100.0 for i in range(R)]
ch = [(w[W + 16 * i + 7] - w[W + 16 * i + 6]) / 100.0 for i in range(R)]
en = [(w[W + 16 * i + 7] - t0) / 100.0 for i in range(R)]
print("scan us: mean %.1f max %.1f | chase+check us: mean %.1f max %.1f | end after t0: max %.1f" % (sum(sc)/R, max(sc), sum(ch)/R, max(ch), max(en)))
print("slowest:", sorted(range(R), key=lambda i: -en[i])[:8], [ (round(sc[i],1), round(ch[i],1)) for i in sorted(range(R), key=lambda i: -en[i])[:8]])
for i in range(64):
    rec = w[W + 16 * i: W + 16 * i + 16]
    if i > 12 and not any(rec[:4]): break
    print(i, "h", rec[0] if rec[0] != NONE else "NONE", "x", rec[1] if rec[1] != NONE else "NONE", "n", rec[2], "ovf", rec[3], "fs", rec[4], "base", w[64 + i], "skip", w[64 + 1024 + i], "ent", w[64 + 2048 + i])
