"""xyws_unmask (k_unmask_range) on the c3-sized batch: R+W GB/s per call over
`reps` calls after `warm` untimed ones, for several warm-up lengths (the
bench's in-run copy ceiling uses 2 + 10).
  usage: unmask_rate.py"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from xynet_amd import websocket as ws
    n = 2147942400
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    buf.fill_(0x5A)
    ctx = ws.Context(0)
    key = (C.c_uint8 * 4)(0x5A, 0xC3, 0x96, 0x21)
    s = torch.cuda.current_stream()
    out = []
    for warm, reps in ((2, 10), (6, 20), (20, 20)):
        for _ in range(warm):
            ctx.L.xyws_unmask(ctx.h, C.c_void_p(buf.data_ptr()), n, key, 0, None, C.c_void_p(s.cuda_stream))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            ctx.L.xyws_unmask(ctx.h, C.c_void_p(buf.data_ptr()), n, key, 0, None, C.c_void_p(s.cuda_stream))
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        out.append({"warm": warm, "reps": reps, "ms": round(ms, 4), "GBps_RW": round(2 * n / (ms * 1e-3) / 1e9, 1)})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
