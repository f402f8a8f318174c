"""One batch split across devices at frame boundaries:
xyws_shard_plan / xyws_shard_plan_frames (host-side planner in libxyws.so,
no device needed) checked against the oracle's stream decode
(oracle/xyws_oracle.c, pinned by the reference's goldens in test_oracle.py).

Properties (CPU):
  * bounds[0] = 0, bounds[n] = len, ascending; every interior bound is a frame
    start of the unsplit decode (or the first start after the carry, or len);
  * balanced within one frame: |bounds[k] - k*len/n| is at most the size of
    the frame holding the target;
  * the shards, each decoded on its own (shard 0 with the carry in, the others
    fresh), give the unsplit decode's bytes, frame list and final carry;
  * the frame-table form gives the same bounds as the byte walk.
The device decode of shards is in tests/test_gpu_parity.py (-m gpu).
"""
import ctypes as C

import numpy as np
import pytest

from xynet_amd import websocket as ws, _lib


def oracle_decode(oracle, buf, carry=None):
    b = buf.copy()
    frames, cout, n = oracle.decode_stream(b, carry_in=carry, cap=max(16, b.size // 2 + 2))
    return b, frames, cout, n


def to_lib_carry(c):
    return _lib.Carry.from_buffer_copy(bytes(c)) if c is not None else None


def check_plan(oracle, buf, n_shards, carry=None):
    bounds = ws.shard_plan(buf, n_shards, carry=to_lib_carry(carry))
    L = buf.size
    assert len(bounds) == n_shards + 1 and bounds[0] == 0 and bounds[-1] == L
    assert all(a <= b for a, b in zip(bounds, bounds[1:]))
    out, frames, cout, n = oracle_decode(oracle, buf, carry)
    starts = {f.frame_off for f in frames if f.frame_off >= 0}
    if cout.hdr_len and L - cout.hdr_len >= 0 and not (carry is not None and n == 0):
        starts.add(L - cout.hdr_len)  # a header cut by the batch end starts a frame too
    starts = sorted(starts)
    ends = starts
    cand = set(starts) | {L}
    first = starts[0] if starts else L
    for k in range(1, n_shards):
        assert bounds[k] in cand, (k, bounds[k])
        assert bounds[k] >= first
        # balance: within the frame holding the target (its start .. next start)
        t = L * k // n_shards
        lo = max([s for s in ends if s <= t], default=0)
        hi = min([s for s in ends if s > t], default=L)
        assert lo <= bounds[k] <= hi or bounds[k] == first, (k, t, bounds[k], lo, hi)
    # each shard decoded alone reproduces the unsplit decode
    pieces, allf, total = [], [], 0
    c_last = None
    for k in range(n_shards):
        a, b = bounds[k], bounds[k + 1]
        part, fr, cout_k, nk = oracle_decode(oracle, buf[a:b], carry if k == 0 else None)
        pieces.append(part)
        allf += [(f.frame_off + a, f.payload_off + a, f.payload_len, bytes(f.key), f.flags, f.hdr_len) for f in fr]
        total += nk
        if b > a or k == 0:
            c_last = (k, cout_k)
        if k < n_shards - 1 and b > a and b < L:
            # an interior shard ends exactly at a frame boundary
            assert cout_k.payload_remaining == 0 and cout_k.hdr_len == 0
    assert np.array_equal(np.concatenate(pieces) if pieces else out, out)
    want = [(f.frame_off, f.payload_off, f.payload_len, bytes(f.key), f.flags, f.hdr_len) for f in frames]
    assert allf == want and total == n
    ck, cc = c_last
    assert (cc.payload_remaining, cc.phase, bytes(cc.key), cc.hdr_len, bytes(cc.hdr)[:cc.hdr_len]) == \
        (cout.payload_remaining, cout.phase, bytes(cout.key), cout.hdr_len, bytes(cout.hdr)[:cout.hdr_len])
    return bounds, frames


@pytest.mark.parametrize("n_shards", [1, 2, 3, 4, 7, 8, 16])
def test_plan_mixed_batch(oracle, n_shards):
    """Config 4's generator (irregular 1 B - 1 MiB frames, fragments, pings) at 24 MiB."""
    tab, n, total = oracle.mixed_table(0x5EED0004, 24 << 20)
    buf = oracle.fill_mixed(tab, n, total, 0x5EED0004)
    bounds, frames = check_plan(oracle, buf, n_shards)
    # the frame-table form agrees with the byte walk
    assert ws.shard_plan_frames(frames, buf.size, n_shards) == bounds


@pytest.mark.parametrize("n_shards", [2, 8])
def test_plan_uniform_exact(oracle, n_shards):
    """Homogeneous frames (config 3 shape, fewer frames): N/n frames per shard."""
    nf, plen = 64, 65536
    buf = oracle.fill_uniform(nf, plen, 0x82, 0x5EED0003)
    fb = plen + 14
    bounds, _ = check_plan(oracle, buf, n_shards)
    assert bounds == [k * nf // n_shards * fb for k in range(n_shards)] + [buf.size]


@pytest.mark.parametrize("cut", [1, 5, 9, 13, 700, 70000])
@pytest.mark.parametrize("n_shards", [2, 5])
def test_plan_with_carry(oracle, cut, n_shards):
    """The batch continues a stream: the carry of the previous batch (a cut
    payload or a cut header) decides where the first frame starts."""
    tab, n, total = oracle.mixed_table(0x5EED0004, 4 << 20)
    stream = oracle.fill_mixed(tab, n, total, 0x5EED0004)
    # cut inside a frame: after `cut` bytes of the frame starting past 1 MiB
    _, frames, _, _ = oracle_decode(oracle, stream)
    f = next(f for f in frames if f.frame_off >= (1 << 20) and f.payload_len + f.hdr_len > cut)
    p = f.frame_off + cut
    first = stream[:p].copy()
    _, carry, _ = oracle.decode_stream(first, cap=len(frames) + 2)
    rest = stream[p:].copy()
    check_plan(oracle, rest, n_shards, carry=carry)


def test_plan_edges(oracle):
    # empty batch
    assert ws.shard_plan(np.zeros(0, np.uint8), 4) == [0, 0, 0, 0, 0]
    # one frame larger than a shard: the other shards are empty
    big = oracle.fill_uniform(1, 1 << 20, 0x82, 7)
    b = ws.shard_plan(big, 4)
    assert b[0] == 0 and b[-1] == big.size and set(b[1:-1]) <= {0, big.size}
    check_plan(oracle, big, 4)
    # a batch ending inside a header and inside a payload
    two = oracle.fill_uniform(8, 1000, 0x81, 9)
    for end in (two.size - 3, two.size - 600, 1004 + 1):
        check_plan(oracle, two[:end].copy(), 3)
    # random bytes (RSV bits, reserved opcodes, any lengths): still the reference's chain
    rng = np.random.default_rng(5)
    junk = rng.integers(0, 256, 200000, dtype=np.uint8)
    for k in (2, 6):
        check_plan(oracle, junk, k)
    L = _lib.load()
    out = (C.c_uint64 * 3)()
    assert L.xyws_shard_plan(None, 0, None, 0, out) == -1
    assert L.xyws_shard_plan(None, 10, None, 2, out) == -1
    # frame table not ascending
    fr = (_lib.Frame * 2)()
    fr[0].frame_off, fr[1].frame_off = 100, 50
    assert L.xyws_shard_plan_frames(fr, 2, 200, 2, out) == -1
