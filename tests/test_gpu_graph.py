"""hipGraph capture of the decode path (xyws_ctx_reserve's promise: after a
reserve, calls allocate nothing and can be captured), replayed and checked
against the oracle.

- A decode with descriptors captured on a stream the context has never seen
  (the reserve's spare slot, include/xyws.h), replayed: bytes, frames, count.
- xyws_unmask captured and replayed an even number of times (its claimed
  tiles' counter is reset in-kernel by the last workgroup, so every replay
  starts from zero): the buffer comes back unchanged, an odd count unmasks.
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
