"""Lattice decoder phase split (XYWS_OPT_STATS): one config batch decoded a few
times, then once with stats; prints microseconds per segment for each phase of
the control lane (tid 0) and of one data lane (tid 64), shader clocks at
2.1 GHz (s_memtime), as one JSON line.
  usage: lat_stats.py [CONFIG] [XOPTS]"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = {16: "ctrl_A_claim_entry0", 17: "ctrl_C_publish_gate", 18: "ctrl_after_D_advance_and_wait_A",
         19: "data_fill", 20: "data_wait_B", 21: "data_table", 22: "data_wait_C", 23: "data_mask_xor_lds",
         24: "data_wait_D", 25: "data_store", 26: "data_wait_A", 28: "ctrl_C_wait_vmcnt"}


def main():
    import torch
    import bench
    from xynet_amd import _lib, websocket as ws
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    xopts = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0
    T = _lib.load_tools()
    buf, info = bench.build_batch(torch, T, cfg, 0, 1)
    dec = ws.frame_decoder(opts=_lib.OPT_LATTICE | xopts)
    if os.environ.get("LAT_STATS_PREV"):  # (a call on another config first: the choice's history)
        pb = bench.build_batch(torch, T, os.environ["LAT_STATS_PREV"], 0, 1)[0]
        ws.frame_decoder(ctx=dec.ctx).decode(pb, cap=0, count=False, carry=False)
        del pb
    dec.ctx.reserve(info["size"], 0)
    for _ in range(6):
        dec.decode(buf, cap=0, count=False, carry=False)
    dec.opts |= _lib.OPT_STATS
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    dec.decode(buf, cap=0, count=False, carry=False)
    e1.record(s)
    torch.cuda.synchronize()
    out = (C.c_uint64 * _lib.NSTATS)()
    dec.ctx.L.xyws_debug_stats(dec.ctx.h, C.c_void_p(s.cuda_stream), out)
    pol = (C.c_uint64 * 5)()
    dec.ctx.L.xyws_debug_policy(dec.ctx.h, C.c_void_p(s.cuda_stream), pol)
    segs = max(1, out[27])
    res = {"config": cfg, "xopts": hex(xopts), "ms_call_with_stats": round(e0.elapsed_time(e1), 4),
           "segments": int(out[27]), "policy": list(pol), "segments_per_workgroup": round(int(out[27]) / 512, 1)}
    for k, n in NAMES.items():
        res["us_per_segment_" + n] = round(out[k] / segs / 2100.0, 3)
    res["us_gate_wait_per_workgroup"] = round(out[29] / max(1, int(sys.argv[3]) if len(sys.argv) > 3 else 256) / 2100.0, 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
