"""hipGraph capture of the decode path (xyws_ctx_reserve's promise: after a
reserve, calls allocate nothing and can be captured), replayed and checked
against the oracle.

- A decode with descriptors captured on a stream the context has never seen
  (the reserve's spare slot, include/xyws.h), replayed: bytes, frames, count.
- A decode with descriptors captured on a stream whose previous calls chose
  the run decoder's 256-thread geometry (echo-sized batches of small frames
  of mixed sizes: four runs per CU), within the reserve.
- xyws_unmask captured and replayed an even number of times (a captured
  unmask takes static tiles: no counter outside the launch): the buffer comes
  back unchanged, an odd count unmasks; a replay on another stream runs
  concurrently with eager unmasks on the capture stream.
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import streams  # noqa: E402


@pytest.mark.gpu
def test_decode_with_descriptors_captured_on_a_new_stream():
    import torch
    from oracle.oracle import Oracle
    from xynet_amd import websocket as ws
    orc = Oracle()
    src = streams.case_bytes("random_frames_200")
    host = np.frombuffer(src, np.uint8).copy()
    ofr, _, on = orc.decode_stream(host)
    ctx = ws.Context(0)
    ctx.reserve(1 << 20, 4096)
    dec = ws.frame_decoder(ctx=ctx)
    buf = torch.frombuffer(bytearray(src), dtype=torch.uint8).cuda()
    orig = buf.clone()
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        r = dec.decode(buf, cap=on + 2, carry=False)  # (within the reserve's 4096 frames)
    # (capture ran nothing: the bytes are untouched)
    torch.cuda.synchronize()
    assert torch.equal(buf, orig)
    for rep in range(3):
        buf.copy_(orig)
        g.replay()
        torch.cuda.synchronize()
        assert buf.cpu().numpy().tobytes() == host.tobytes(), rep
        assert r.nframes == on
        got = [(f.frame_off, f.payload_off, f.payload_len, bytes(f.key), f.flags, f.hdr_len, f.status)
               for f in r.frames()]
        want = [(f.frame_off, f.payload_off, f.payload_len, bytes(f.key), f.flags, f.hdr_len, f.status)
                for f in ofr]
        assert got == want, rep
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,phase", [(1 << 22, 0), ((1 << 22) + 13, 3)])
def test_unmask_captured_and_replayed(n, phase):
    import torch
    from xynet_amd import websocket as ws
    g0 = torch.Generator().manual_seed(5)
    data = torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g0).cuda()
    orig = data.clone()
    mask = 0x1F2E3D4C
    view = data[5:]  # (misaligned start)
    ws.context(0).reserve(n + 64)  # (the claim counter of a stream new to the context)
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        ws.websocket_mask(view, mask, phase)
    torch.cuda.synchronize()
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(data, orig)
    g.replay()
    torch.cuda.synchronize()
    kb = np.frombuffer(mask.to_bytes(4, "little"), np.uint8)
    want = orig.cpu().numpy().copy()
    idx = (phase + np.arange(n - 5)) % 4
    want[5:] ^= kb[idx]
    assert np.array_equal(data.cpu().numpy(), want)


@pytest.mark.gpu
def test_decode_captured_after_mid_geometry_calls():
    """the reserve must cover the 256-thread geometry's run count
    (ncu * 4 runs on 16 KiB segments), which the decoder choice gives a
    stream after calls of small frames of mixed sizes."""
    import torch
    from oracle.oracle import Oracle
    from xynet_amd import websocket as ws
    orc = Oracle()
    rng = streams.SplitMix(0x6D1D)
    b = bytearray()
    while len(b) < (4 << 20) - 1100:
        b += streams.frame(rng, 0x81, rng.next() % 1001)
    src = bytes(b)
    host = np.frombuffer(src, np.uint8).copy()
    ofr, _, on = orc.decode_stream(host, cap=len(src) // 6 + 2)
    ctx = ws.Context(0)
    ctx.reserve(4 << 20, 16384)
    dec = ws.frame_decoder(ctx=ctx)
    orig = torch.frombuffer(bytearray(src), dtype=torch.uint8).cuda()
    buf = orig.clone()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(2):  # (eager: the policy words now say small frames of mixed sizes)
            buf.copy_(orig)
            r = dec.decode(buf, cap=on + 2, carry=False)
            assert r.nframes == on
    torch.cuda.synchronize()
    pol = (__import__("ctypes").c_uint64 * 5)()
    assert ctx.L.xyws_debug_policy(ctx.h, __import__("ctypes").c_void_p(s.cuda_stream), pol) == 0
    assert pol[3] < 2048 and pol[2] != pol[3], list(pol)
    g = torch.cuda.CUDAGraph()
    buf.copy_(orig)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        r = dec.decode(buf, cap=on + 2, carry=False)
    torch.cuda.synchronize()
    for rep in range(2):
        buf.copy_(orig)
        g.replay()
        torch.cuda.synchronize()
        assert buf.cpu().numpy().tobytes() == host.tobytes(), rep
        assert r.nframes == on
        got = [(f.frame_off, f.payload_off, f.payload_len, bytes(f.key), f.flags, f.hdr_len, f.status)
               for f in r.frames()]
        want = [(f.frame_off, f.payload_off, f.payload_len, bytes(f.key), f.flags, f.hdr_len, f.status)
                for f in ofr]
        assert got == want, rep
    ctx.close()


@pytest.mark.gpu
def test_unmask_replay_concurrent_with_eager_unmask_on_the_capture_stream():
    """A captured unmask replayed on stream B while eager unmasks run on the
    capture stream A: the replay shares no counter with them."""
    import torch
    from xynet_amd import websocket as ws
    n = 96 << 20
    g0 = torch.Generator().manual_seed(9)
    a = torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g0).cuda()
    b = torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g0).cuda()
    a0, b0 = a.clone(), b.clone()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(sa):
        ws.websocket_mask(b, 0x01020304, 0)  # (eager on A first: A's slot and counter exist)
        ws.websocket_mask(b, 0x01020304, 0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=sa):
        ws.websocket_mask(a, 0xA5C3E1F0, 1)
    torch.cuda.synchronize()
    for _ in range(3):
        with torch.cuda.stream(sb):
            g.replay()
            g.replay()
        with torch.cuda.stream(sa):
            ws.websocket_mask(b, 0x01020304, 0)
            ws.websocket_mask(b, 0x01020304, 0)
    torch.cuda.synchronize()
    assert torch.equal(a, a0)
    assert torch.equal(b, b0)
