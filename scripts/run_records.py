"""Run decoder per-run timeline (debug aid, XYWS_OPT_STATS): one config batch
decoded with the run decoder after warm-up calls, then once with stats; from
the run records (s_memrealtime, 100 MHz): each run's prologue (entry scan),
main phase and end after the first run's start, and its scan distance (entry
minus range start). Prints one JSON line.
  usage: run_records.py [CONFIG] [XOPTS]"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from xynet_amd import _lib, websocket as ws
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    xopts = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0
    T = _lib.load_tools()
    buf, info = bench.build_batch(torch, T, cfg, 0, 1)
    dec = ws.frame_decoder(opts=_lib.OPT_RUNS | xopts)
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
    nrec = 2048
    out = (C.c_uint64 * (nrec * _lib.R_WORDS))()
    n = dec.ctx.L.xyws_debug_records(dec.ctx.h, C.c_void_p(s.cuda_stream), out, nrec)
    W = _lib.R_WORDS
    R_H, R_T0, R_T1, R_T2 = 0, 25, 26, 27
    NONE = (1 << 64) - 1
    runs = []
    for f in range(0, n, 2):
        t0, t1, t2 = out[f * W + R_T0], out[f * W + R_T1], out[f * W + R_T2]
        if not t0 or not t2 or t2 < t0:
            continue
        runs.append((f // 2, t0, t1, t2, out[f * W + R_H]))
    if not runs:
        print(json.dumps({"config": cfg, "error": "no records"}))
        return
    tmin = min(r[1] for r in runs)
    size = info["size"]
    rb = (size + len(runs) - 1) // len(runs)
    pro = [(r[2] - r[1]) / 100.0 for r in runs]
    mainp = [(r[3] - r[2]) / 100.0 for r in runs]
    end = [(r[3] - tmin) / 100.0 for r in runs]
    start = [(r[1] - tmin) / 100.0 for r in runs]
    dist = [((r[4] - r[0] * rb) / 1024.0) if r[4] != NONE else -1 for r in runs]
    slow = sorted(range(len(runs)), key=lambda i: -end[i])[:8]
    res = {"config": cfg, "xopts": hex(xopts), "ms_call_with_stats": round(e0.elapsed_time(e1), 4), "runs": len(runs),
           "start_us_max": round(max(start), 1),
           "prologue_us": {"mean": round(sum(pro) / len(pro), 1), "max": round(max(pro), 1)},
           "main_us": {"mean": round(sum(mainp) / len(mainp), 1), "max": round(max(mainp), 1)},
           "end_us": {"mean": round(sum(end) / len(end), 1), "max": round(max(end), 1)},
           "scan_kib": {"mean": round(sum(d for d in dist if d >= 0) / max(1, sum(1 for d in dist if d >= 0)), 1),
                        "max": round(max(dist), 1)},
           "slowest": [{"run": runs[i][0], "start": round(start[i], 1), "pro": round(pro[i], 1),
                        "main": round(mainp[i], 1), "end": round(end[i], 1), "scan_kib": round(dist[i], 1)}
                       for i in slow]}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
