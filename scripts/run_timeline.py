#!/usr/bin/env python3
"""Per-run timeline of one fused stream decode (diagnostic, not product).

Decodes a bench batch with the stats option, then reads every run's record
(start, end of prologue, end: s_memrealtime, 100 MHz) and prints the spread
of run start/prologue/end times, i.e. how much of a call is spent with some
CUs idle. Usage: python scripts/run_timeline.py [c3|c2|c1|c4] [extra XYWS_OPT bits]
"""
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from xynet_amd import _lib, websocket as ws
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    xopts = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0
    T = _lib.load_tools()
    buf, info = bench.build_batch(torch, T, cfg, 0, 1)
    dec = ws.frame_decoder(opts=xopts)
    stream = torch.cuda.current_stream()
    for _ in range(3):
        dec.decode(buf, cap=0, count=False, carry=False)
    dec.opts |= _lib.OPT_STATS
    dec.decode(buf, cap=0, count=False, carry=False)
    torch.cuda.synchronize()
    R = (C.c_uint64 * (1024 * _lib.R_WORDS))()
    n = dec.ctx.L.xyws_debug_records(dec.ctx.h, C.c_void_p(stream.cuda_stream), R, 1024)
    recs = [list(R[i * _lib.R_WORDS:(i + 1) * _lib.R_WORDS]) for i in range(n)]
    t0s = [r[25] for r in recs if r[25]]
    base = min(t0s)
    rows = []
    for i, r in enumerate(recs):
        if not r[25]:
            continue
        rows.append(dict(run=i // 2, piece=i & 1, xcc=r[29], start=(r[25] - base) / 100.0,
                         prologue=(r[26] - r[25]) / 100.0 if r[26] else None,
                         end=(r[27] - base) / 100.0 if r[27] else None))
    ends = [x["end"] for x in rows if x["end"] is not None]
    pros = [x["prologue"] for x in rows if x["prologue"] is not None]
    starts = [x["start"] for x in rows]
    out = {"config": cfg, "runs": len(rows),
           "start_us": [round(min(starts), 2), round(statistics.mean(starts), 2), round(max(starts), 2)],
           "prologue_us": [round(min(pros), 2), round(statistics.mean(pros), 2), round(max(pros), 2)],
           "end_us": [round(min(ends), 2), round(statistics.mean(ends), 2), round(statistics.median(ends), 2),
                      round(max(ends), 2)],
           "latest_runs": sorted(rows, key=lambda x: -(x["end"] or 0))[:8]}
    by_xcc = {}
    for x in rows:
        if x["end"] is not None and not x["piece"]:
            by_xcc.setdefault(x["xcc"], []).append(x["end"])
    out["end_us_by_xcc"] = {k: [len(v), round(min(v), 1), round(statistics.mean(v), 1), round(max(v), 1)]
                            for k, v in sorted(by_xcc.items())}
    # which part of a run's range: the end time against the run index mod 8 / 32
    by_mod = {}
    for x in rows:
        if x["end"] is not None and not x["piece"]:
            by_mod.setdefault(x["run"] % 8, []).append(x["end"])
    out["end_us_by_run_mod8"] = {k: round(statistics.mean(v), 1) for k, v in sorted(by_mod.items())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
