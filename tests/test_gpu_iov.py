"""xyws_decode_stream_iov (include/xyws.h) against the oracle (gpu).

A recv fills a multi-buffer buffer_sequence (include/xynet/buffer.h:94-110,
socket/impl/recv_all.h:99-121); the pieces are one stream. Every case splits
a stream into pieces of random lengths (0-length pieces included) at random
alignments, decodes the sequence in one call, and compares each piece's
bytes, the descriptor table (offsets across the pieces) and the carry with
the oracle's decode of the concatenation; then a stream cut across two
sequences (the carry between calls), equal frames (the lattice decoder), and
the limits (XYWS_IOV_MAX pieces; more is refused). Without descriptors the
pieces may be decoded in place one by one, the carry chained between them
on the device (XYWS_OPT_IOV_PIECES forces it: every case again in that
mode, count, bytes and carry)."""
import numpy as np
import pytest

import streams
from test_gpu_parity import carry_list, dev_bytes, frames_list, host, torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ws():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from xynet_amd import websocket
    return websocket


def pieces_of(src, rng, n):
    cuts = sorted(set([0, len(src)] + [rng.below(len(src) + 1) for _ in range(n - 1)]))
    # (a repeated cut: a 0-length piece)
    if n > 2:
        cuts.insert(1, cuts[1])
    return [src[a:b] for a, b in zip(cuts[:-1], cuts[1:])]


OPT_IOV_PIECES = 0x10000000  # xyws_stream.h: the pieces in place one by one (no descriptors)


def decode_seq(ws, oracle, dec, seq, carry_in, rng, desc=True):
    views, wholes, offs = [], [], []
    for p in seq:
        off = rng.below(16)
        v, w = dev_bytes(p, off)
        views.append(v)
        wholes.append((w, off, len(p)))
    cat = b"".join(seq)
    ob = np.frombuffer(cat, np.uint8).copy() if cat else np.zeros(0, np.uint8)
    ofr, carry, on = oracle.decode_stream(ob, carry_in=carry_in)
    r = dec.decode_iov(views, cap=on + 2 if desc else 0)
    assert r.nframes == on
    got = b"".join(host(v) for v in views)
    assert got == ob.tobytes()
    for w, off, n in wholes:
        out = host(w)
        assert out[:off] == b"\xa5" * off and out[off + n:] == b"\xa5" * 32  # (nothing outside the pieces)
    if desc:
        assert frames_list(r.frames(), True) == frames_list(ofr, True)
    assert carry_list(dec.carry()) == carry_list(carry)
    return carry


@pytest.mark.parametrize("name", ["random_frames_3", "random_frames_50", "random_frames_300", "lengths"])
@pytest.mark.parametrize("npieces", [1, 2, 5, 17])
def test_sequence_matches_the_concatenation(ws, oracle, name, npieces):
    src = streams.case_bytes(name)
    rng = streams.SplitMix(len(src) * 31 + npieces)
    dec = ws.frame_decoder()
    decode_seq(ws, oracle, dec, pieces_of(src, rng, npieces), None, rng)


@pytest.mark.parametrize("name", ["random_frames_3", "random_frames_50", "random_frames_300", "lengths"])
@pytest.mark.parametrize("npieces", [2, 5, 17])
def test_pieces_in_place(ws, oracle, name, npieces):
    src = streams.case_bytes(name)
    rng = streams.SplitMix(len(src) * 37 + npieces)
    dec = ws.frame_decoder(opts=OPT_IOV_PIECES)
    decode_seq(ws, oracle, dec, pieces_of(src, rng, npieces), None, rng, desc=False)
    # (a stream across two sequences: the carry between calls, the count per call)
    dec2 = ws.frame_decoder(opts=OPT_IOV_PIECES)
    cut = rng.below(len(src))
    c = decode_seq(ws, oracle, dec2, pieces_of(src[:cut], rng, npieces), None, rng, desc=False)
    decode_seq(ws, oracle, dec2, pieces_of(src[cut:], rng, npieces), c, rng, desc=False)


def test_stream_across_two_sequences(ws, oracle):
    """The carry between calls: a frame or header cut by the first sequence's
    end continues in the second."""
    src = streams.case_bytes("random_frames_200")
    rng = streams.SplitMix(7)
    for it in range(6):
        cut = rng.below(len(src))
        dec = ws.frame_decoder()
        c = decode_seq(ws, oracle, dec, pieces_of(src[:cut], rng, 4), None, rng)
        decode_seq(ws, oracle, dec, pieces_of(src[cut:], rng, 3), c, rng)


def test_equal_frames_take_the_lattice_decoder(ws, oracle):
    rng = streams.SplitMix(11)
    src = bytearray()
    for _ in range(3000):
        src += streams.frame(rng, 0x82, 500)
    src = bytes(src)
    dec = ws.frame_decoder()
    c = None
    for _ in range(3):  # (one stream: the frame count carries on)
        c = decode_seq(ws, oracle, dec, pieces_of(src, rng, 9), c, rng)


def test_piece_limit(ws, oracle):
    src = streams.case_bytes("random_frames_50")
    rng = streams.SplitMix(3)
    n = 64  # XYWS_IOV_MAX
    cuts = sorted(rng.below(len(src)) for _ in range(n - 1))
    seq = [src[a:b] for a, b in zip([0] + cuts, cuts + [len(src)])]
    dec = ws.frame_decoder()
    decode_seq(ws, oracle, dec, seq, None, rng)
    views = [dev_bytes(b"\x82\x80abcd", 0)[0] for _ in range(n + 1)]
    with pytest.raises(Exception):
        dec.decode_iov(views)  # (XYWS_ERR_INVALID)


def test_captured_after_reserve_iov(ws, oracle):
    """xyws_ctx_reserve + xyws_ctx_reserve_iov, then an iov decode captured
    into a hipGraph on a stream new to the context (the reserve's spare
    slot): the capture allocates nothing; every replay decodes the pieces in
    place as the oracle decodes their concatenation."""
    src = streams.case_bytes("random_frames_200")
    rng = streams.SplitMix(0x10F)
    seq = pieces_of(src, rng, 7)
    host = np.frombuffer(src, np.uint8).copy()
    _, _, on = oracle.decode_stream(host)
    ctx = ws.Context(0)
    ctx.reserve(len(src) + 64, 4096)
    ctx.reserve_iov(len(src) + 64)
    dec = ws.frame_decoder(ctx=ctx)
    views = [torch.frombuffer(bytearray(b if b else b"\0"), dtype=torch.uint8).cuda()[: len(b)] for b in seq]
    origs = [v.clone() for v in views]
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        r = dec.decode_iov(views, cap=0, carry=False)
    torch.cuda.synchronize()
    for rep in range(3):
        for v, o in zip(views, origs):
            v.copy_(o)
        g.replay()
        torch.cuda.synchronize()
        got = b"".join(v.cpu().numpy().tobytes() for v in views)
        assert got == host.tobytes(), rep
        assert r.nframes == on, rep
    ctx.close()
