"""The lattice decoder (xynet_amd/csrc/xyws_lattice.h) against the oracle (gpu).

Frame boundaries are a linked list (websocket_frame_header.h:305-385); for a
batch of equal frames it is the lattice X0 + k*F, which the lattice decoder
checks at every point in parallel, handing the batch from the first point off
the lattice to the run decoder (a redirect in the same stream). Every case is
decoded with the lattice forced (XYWS_OPT_LATTICE) in the production geometry
and in 1 KiB segments (many segments, look-backs and straddling headers), at
misaligned offsets, whole and split with carry, and compared byte for byte,
frame for frame and carry for carry with the pinned restatement:

* regular batches of every header form (F = 128 .. 200 KiB), the last frame
  whole, cut in its payload or cut in its header;
* one size change at the first, a middle and the last frame (the redirect);
* equal F from different header forms (non-minimal lengths: H varies);
* a batch that starts inside a carried frame or a carried header;
* frames under LAT_FMIN and a batch inside one frame (not applicable: the run
  decoder takes all of it);
* descriptor capacities below the frame count.
"""
import numpy as np
import pytest

import streams
from test_gpu_parity import carry_list, dev_bytes, frames_list, host, torch
from test_gpu_choice import _policy

pytestmark = pytest.mark.gpu

OPT_LATTICE = 0x400
OPT_SMALL = 0x200
OPT_TEST_LATSPEC = 0x10  # every store speculative: a broken lattice is undone by the end-of-work check
OPT_TEST_LATDUMP = 0x20  # no workgroup undoes its own stores at its end: every list goes to the finisher
MODES = {"lat": {"opts": OPT_LATTICE}, "lat1k": {"opts": OPT_LATTICE | OPT_SMALL},
         "lat_blind": {"opts": OPT_LATTICE | OPT_TEST_LATSPEC},
         "lat1k_blind": {"opts": OPT_LATTICE | OPT_SMALL | OPT_TEST_LATSPEC},
         "lat_blind_dump": {"opts": OPT_LATTICE | OPT_TEST_LATSPEC | OPT_TEST_LATDUMP},
         "lat1k_blind_dump": {"opts": OPT_LATTICE | OPT_SMALL | OPT_TEST_LATSPEC | OPT_TEST_LATDUMP}}


@pytest.fixture(scope="module")
def ws():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from xynet_amd import websocket
    return websocket


def regular(seed, plen, n, b0=0x82, form=None, tail=None):
    """n masked frames of plen payload bytes; tail: None, ("payload", k) or
    ("header", k): the stream cut k bytes into the last frame."""
    rng = streams.SplitMix(seed)
    out = bytearray()
    for _ in range(n):
        out += streams.frame(rng, b0, plen, form=form)
    if tail:
        kind, k = tail
        h = len(streams.header(b0, plen, b"\0" * 4, form))
        last = streams.frame(rng, b0, plen, form=form)
        out += last[:k] if kind == "header" else last[:h + k]
    return bytes(out)


def decode_pieces(ws, oracle, src, cuts, mode, offset=0, cap_frac=1.0):
    dec = ws.frame_decoder(**MODES[mode])
    carry = None
    for a, b in zip(cuts[:-1], cuts[1:]):
        piece = src[a:b]
        view, whole = dev_bytes(piece, offset)
        ob = np.frombuffer(piece, np.uint8).copy() if piece else np.zeros(0, np.uint8)
        ofr, carry, on = oracle.decode_stream(ob, carry_in=carry)
        cap = int(on * cap_frac) + (2 if cap_frac >= 1 else 0)
        r = dec.decode(view, cap=cap)
        assert r.nframes == on, (mode, a, b)
        out = host(whole)
        assert out[:offset] == b"\xa5" * offset and out[offset + len(piece):] == b"\xa5" * 32
        assert host(view) == ob.tobytes(), (mode, a, b)
        got = frames_list(r.frames(), True)
        assert got == frames_list(ofr[:min(on, cap)], True), (mode, a, b)
        assert carry_list(dec.carry()) == carry_list(carry), (mode, a, b)


PLENS = [122, 123, 200, 256, 1000, 4096, 65535, 65536, 200000]


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("plen", PLENS)
def test_regular_batches(ws, oracle, mode, plen):
    n = max(3, min(400, (3 << 20) // (plen + 14)))
    for tail in (None, ("payload", 1), ("payload", plen - 1), ("header", 1), ("header", 5)):
        src = regular(plen * 7 + 1, plen, n, tail=tail)
        for off in (0, 3):
            decode_pieces(ws, oracle, src, [0, len(src)], mode, off)


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("plen", [200, 4096, 65536])
@pytest.mark.parametrize("where", ["first", "middle", "last"])
def test_size_change_redirects(ws, oracle, mode, plen, where):
    """The first frame off the lattice: everything before it is the lattice
    decoder's, the rest the run decoder's (frame count, ordinals and offsets
    continued)."""
    n = max(4, min(300, (2 << 20) // (plen + 14)))
    j = {"first": 1, "middle": n // 2, "last": n - 1}[where]
    rng = streams.SplitMix(plen + j)
    src = bytearray()
    for i in range(n):
        p = plen if i < j else (plen + 17 if i == j else plen)
        src += streams.frame(rng, 0x82, p)
    src = bytes(src)
    decode_pieces(ws, oracle, src, [0, len(src)], mode, 1)
    decode_pieces(ws, oracle, src, [0, len(src)], mode, 0, cap_frac=0.6)


@pytest.mark.parametrize("mode", list(MODES))
def test_equal_size_from_different_header_forms(ws, oracle, mode):
    """F = H + P equal while H differs (non-minimal 16-bit lengths, accepted
    by the reference parser): every frame's own header decides its payload."""
    rng = streams.SplitMix(99)
    src = bytearray()
    for i in range(600):
        if rng.below(3) == 0:
            src += streams.frame(rng, 0x82, 118, form=16)   # H = 8, P = 118
        else:
            src += streams.frame(rng, 0x82, 120)            # H = 6, P = 120
    src = bytes(src)
    decode_pieces(ws, oracle, src, [0, len(src)], mode, 0)
    decode_pieces(ws, oracle, src, [0, len(src)], mode, 7)


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("plen", [300, 65536])
def test_split_batches_with_carry(ws, oracle, mode, plen):
    """Batches that start inside a carried frame or a carried header."""
    n = max(6, min(200, (2 << 20) // (plen + 14)))
    src = regular(plen + 3, plen, n)
    fsz = len(src) // n
    rng = streams.SplitMix(plen)
    for it in range(6):
        cuts = sorted(set([0, len(src)] + [rng.below(len(src)) for _ in range(2)] +
                          [fsz * (1 + rng.below(n - 1)) + rng.below(14)]))
        decode_pieces(ws, oracle, src, cuts, mode, it % 4)


@pytest.mark.parametrize("mode", list(MODES))
def test_not_applicable_batches(ws, oracle, mode):
    """Frames under LAT_FMIN (128 B), a batch inside one frame, a batch that
    opens in a cut header: the run decoder decodes all of it."""
    small = regular(5, 60, 3000)
    decode_pieces(ws, oracle, small, [0, len(small)], mode, 0)
    big = regular(6, 1 << 20, 1)
    decode_pieces(ws, oracle, big, [0, 5, 70000, 300001, len(big)], mode, 0)
    decode_pieces(ws, oracle, big, [0, 3, 9, len(big)], mode, 2)


@pytest.mark.parametrize("mode", list(MODES))
def test_irregular_streams(ws, oracle, mode):
    """Random frame soups (the first size change at frame 1)."""
    for n in (3, 50, 300):
        src = streams.case_bytes(f"random_frames_{n}")
        decode_pieces(ws, oracle, src, [0, len(src)], mode, 0)
    src = streams.case_bytes("random_frames_200")
    decode_pieces(ws, oracle, src, [0, len(src) // 3, len(src)], mode, 5)


def _big_regular(seed, plen, nbytes, change_at=None):
    """A regular batch of about nbytes (frames of plen payload bytes, minimal
    16-bit form, random keys and payloads, numpy-built); frame change_at (from
    the end when negative) has plen + 17 payload bytes."""
    r = np.random.default_rng(seed)
    n = nbytes // (plen + 8)
    fr = r.integers(0, 256, size=(n, plen + 8), dtype=np.uint8)
    fr[:, 0] = 0x82
    fr[:, 1] = 0x80 | 126
    fr[:, 2] = plen >> 8
    fr[:, 3] = plen & 0xFF
    if change_at is None:
        return fr.reshape(-1).copy(), n
    j = change_at % n
    odd = r.integers(0, 256, size=plen + 17 + 8, dtype=np.uint8)
    odd[:4] = [0x82, 0x80 | 126, (plen + 17) >> 8, (plen + 17) & 0xFF]
    return np.concatenate([fr[:j].reshape(-1), odd, fr[j + 1:].reshape(-1)]), n


@pytest.mark.parametrize("change_at", [None, -3])
def test_speculation_list_overflow_hands_over(ws, oracle, change_at):
    """The lattice decoder's speculative-store list (LAT_SLIST = 512 segments
    per workgroup, xyws_lattice.h): past it a workgroup raises the failing
    point to the frame before its segment and the run decoder takes the rest
    (stores past that point undone). In 1 KiB segments (64 workgroups) a
    regular batch above 32 MiB reaches it: 40 MiB, with and without a size
    change near its end. Bytes, count, the whole descriptor table and the
    carry against the oracle; the lattice did not finish the call (the run
    decoder took the tail: policy word 4 != 3)."""
    from test_gpu_parity import decoder_policy
    src, n = _big_regular(0x5A17 + (change_at or 0), 4096, 40 << 20, change_at)
    ob = src.copy()
    oraw, ocarry, on = oracle.decode_stream_raw(ob, on_cap := n + 2)
    t = torch.from_numpy(src.copy()).cuda()
    dec = ws.frame_decoder(**MODES["lat1k"])
    r = dec.decode(t, cap=on_cap)
    assert r.nframes == on
    assert dec.ctx.last_device_error() == 0
    assert oracle.digest(t.cpu().numpy()) == oracle.digest(ob)
    assert oracle.frames_digest(r.frames_t[: on * 32].cpu().numpy()) == oracle.frames_digest(oraw)
    assert carry_list(dec.carry()) == carry_list(ocarry)
    assert decoder_policy(dec)[4] != 3, decoder_policy(dec)


def test_lattice_then_irregular_then_lattice(ws, oracle):
    """The decoder choice without forcing: regular batches take the lattice,
    an irregular one after them is redirected at its first size change, the
    next irregular one takes the run decoder, and a regular one after that
    the run decoder once more (the choice follows the previous call), then the
    lattice again (policy word 4: 3 = lattice)."""
    dec = ws.frame_decoder()
    reg = regular(1, 4096, 500)
    irr = streams.case_bytes("random_frames_300")
    used = []
    for src in (reg, reg, irr, irr, reg, reg):
        view, _ = dev_bytes(src)
        ob = np.frombuffer(src, np.uint8).copy()
        ofr, _, on = oracle.decode_stream(ob)
        r = dec.decode(view, cap=on + 2, carry=False)
        assert r.nframes == on
        assert host(view) == ob.tobytes()
        assert frames_list(r.frames(), True) == frames_list(ofr, True)
        used.append(_policy(dec)[4])
    assert used[1] == 3 and used[3] != 3 and used[4] != 3 and used[5] == 3  # (call 0 follows the stream's past)
