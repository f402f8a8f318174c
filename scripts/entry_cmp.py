"""Debug aid: the run decoder's per-run entries (R_H) of one config batch for
the given xopts variants, printed side by side (first N runs) with the
frame count of each variant.
  usage: entry_cmp.py CONFIG N XOPTS..."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from xynet_amd import _lib, websocket as ws
    cfg, nshow = sys.argv[1], int(sys.argv[2])
    T = _lib.load_tools()
    buf, info = bench.build_batch(torch, T, cfg, 0, 1)
    cols = []
    for xs in sys.argv[3:]:
        x = int(xs, 0)
        dec = ws.frame_decoder(opts=_lib.OPT_RUNS | x)
        for _ in range(3):   # (the policy words: the bigscan hint follows the previous call)
            r = dec.decode(buf, cap=0, count=True, carry=False)
        nf = r.nframes
        out = (C.c_uint64 * (2048 * _lib.R_WORDS))()
        s = torch.cuda.current_stream()
        n = dec.ctx.L.xyws_debug_records(dec.ctx.h, C.c_void_p(s.cuda_stream), out, 2048)
        cols.append((xs, nf, [out[f * _lib.R_WORDS] for f in range(0, n, 2)]))
    print("frames", [(c[0], c[1]) for c in cols], "expected", info["nframes"])
    NONE = (1 << 64) - 1
    for i in range(nshow):
        row = [("NONE" if c[2][i] == NONE else c[2][i]) for c in cols]
        flag = "" if len(set(row)) == 1 else "  <-- differs"
        print(i, row, flag)


if __name__ == "__main__":
    main()
