"""xyws_decode_stream_iov's rate on a multi-piece sequence: a
config batch cut at random offsets into PIECES separate device buffers (one
recv's buffer_sequence, include/xynet/buffer.h:94-110), decoded as ONE stream
(gather into the staging buffer, decode, scatter back), against
xyws_decode_stream on the same bytes in one buffer. Payload GiB/s per call
(HIP events over REPS calls after warm-up calls; an even number of calls
before the checks, so the pieces end as they started, plus one odd call
checked against the reference's output digest). One JSON line.
  usage: iov_rate.py [CONFIG] [PIECES] [REPS]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import torch
    from test_gpu_parity import tools_batch, dev_digest
    from xynet_amd import websocket as ws
    name = sys.argv[1] if len(sys.argv) > 1 else "c1_text_4k"
    npieces = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    buf, c = tools_batch(name)
    n = buf.numel()
    g = torch.Generator().manual_seed(npieces)
    cuts = sorted(torch.randint(1, n, (npieces - 1,), generator=g).tolist())
    bounds = list(zip([0] + cuts, cuts + [n]))
    pieces = [buf[a:b].clone() for a, b in bounds]
    dec = ws.frame_decoder()
    dec.ctx.reserve(n + 64, 0)
    dec.ctx.reserve_iov(n + 64)
    s = torch.cuda.current_stream()

    def timed(fn):
        for _ in range(4):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    from xynet_amd import _lib  # noqa: F401
    dec.opts = 0x20000000  # XYWS_OPT_IOV_STAGE: gather, decode, scatter
    ms_stage = timed(lambda: dec.decode_iov(pieces, cap=0, count=False, carry=False))
    dec.opts = 0x10000000  # XYWS_OPT_IOV_PIECES: the pieces in place, carry chained
    ms_iov = timed(lambda: dec.decode_iov(pieces, cap=0, count=False, carry=False))
    dec.opts = 0
    ms_one = timed(lambda: dec.decode(buf, cap=0, count=False, carry=False))
    # (4 + reps calls each: an even count when reps is even) one more iov call
    # (in pieces): unmasked
    assert (4 + reps) % 2 == 0
    dec.opts = 0x10000000
    r = dec.decode_iov(pieces, cap=0, count=True, carry=False)
    whole = torch.cat(pieces)
    ok = dev_digest(whole) == c["out_digest"] and r.nframes == c["decoded_frames"]
    res = {"config": name, "pieces": npieces, "batch_bytes": n, "ms_stage": round(ms_stage, 4),
           "ms_pieces": round(ms_iov, 4), "ms_contiguous": round(ms_one, 4),
           "ratio_stage": round(ms_stage / ms_one, 3), "ratio_pieces": round(ms_iov / ms_one, 3),
           "gbps_stage_batch": round(n / (ms_stage * 1e-3) / 1e9, 1),
           "gbps_pieces_batch": round(n / (ms_iov * 1e-3) / 1e9, 1),
           "gbps_contiguous_batch": round(n / (ms_one * 1e-3) / 1e9, 1), "parity": ok}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
