"""The decoder choice across configs on one stream (tests/test_gpu_choice.py::
test_decoder_choice_follows_the_frames, timed): c3, c3, c4, c4, c4, each call's
HIP-event time and the decoder that served it. Run under
`rocprofv3 --kernel-trace` to split a call into its kernels.
  usage: choice_trace.py [SEQ]   (SEQ: comma-separated config names)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import ctypes as C
    import torch
    import bench
    from xynet_amd import _lib, websocket as ws
    seq = (sys.argv[1] if len(sys.argv) > 1 else "c3,c3,c4,c4,c4").split(",")
    T = _lib.load_tools()
    dec = ws.frame_decoder()
    bufs = {}
    s = torch.cuda.current_stream()
    out = []
    for cfg in seq:
        if cfg not in bufs:
            bufs.clear()
            torch.cuda.empty_cache()
            bufs[cfg] = bench.build_batch(torch, T, cfg, 0, 1)[0]
        buf = bufs[cfg]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        dec.decode(buf, cap=0, count=False, carry=False)
        e1.record(s)
        torch.cuda.synchronize()
        pol = (C.c_uint64 * 5)()
        dec.ctx.L.xyws_debug_policy(dec.ctx.h, C.c_void_p(s.cuda_stream), pol)
        out.append({"config": cfg, "ms": round(e0.elapsed_time(e1), 4), "decoder": int(pol[4]),
                    "fsmin": int(pol[2]), "fsmax": int(pol[3])})
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
