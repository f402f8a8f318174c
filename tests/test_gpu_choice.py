"""The decoder choice of xyws_decode_stream (stream_decode_fused), through the
C-ABI: which decoder serves a call follows what the previous call on the same
stream found (the policy words its finisher publishes), and every call's bytes,
count and carry are the reference's whichever decoder ran
(tests/golden/configs.json, from the real reference headers).
"""
import ctypes as C

import pytest

from test_gpu_parity import dev_digest, tools_batch

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def ws():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from xynet_amd import websocket
    return websocket


def _policy(dec):
    out = (C.c_uint64 * 5)()
    stream = torch.cuda.current_stream()
    assert dec.ctx.L.xyws_debug_policy(dec.ctx.h, C.c_void_p(stream.cuda_stream), out) == 0
    return list(out)


def _lat_counters(dec):
    """xyws_debug_lattice: {device policy word, lattice calls handed whole to
    the run decoder on it, ... by the prologue's checks, lattice calls whose
    segment loops ran in 75 KiB segments, in 120 KiB segments} (cumulative per
    stream slot). Synchronizes the device."""
    out = (C.c_uint64 * 5)()
    stream = torch.cuda.current_stream()
    assert dec.ctx.L.xyws_debug_lattice(dec.ctx.h, C.c_void_p(stream.cuda_stream), out) == 0
    return list(out)


def test_decoder_choice_follows_the_frames(ws):
    """The decoder choice (stream_decode_fused): the lattice decoder first when
    the previous call on the stream found frames of one size (>= 128 B, policy
    word 4 = 3), the run decoder otherwise (0, or
    2 in 512-thread workgroups after regular frames under 2 KiB). An irregular
    batch after regular ones goes to the lattice decoder, which checks lattice
    points 1 and 2 before anything else and hands the whole batch to the run
    decoder: its time stays that of the run decoder alone (the decoder-choice
    cliff of round 3 was 7x: the retired sweep decoder scanning every segment;
    round 4's lattice attempt cost 54 us). Every call is checked against the
    reference's digests, whichever decoder ran."""
    from xynet_amd import _lib
    # (calls 4, 5: the run decoder with the hints a c3 history gives it, the
    # one-pass entry scan off, so that they time what call 3 runs after its
    # hand-over)
    alone = _lib.OPT_RUNS | _lib.OPT_NO_BIGSCAN
    seq = [("c3_bin_64k", 0), ("c3_bin_64k", 0), ("c3_bin_64k", 0), ("c4_mixed", 0), ("c4_mixed", alone),
           ("c4_mixed", alone), ("c4_mixed", 0), ("c4_mixed", 0), ("c2_bin_256", 0), ("c2_bin_256", 0),
           ("c3_bin_64k", _lib.OPT_RUNS), ("c3_bin_64k", 0), ("c3_bin_64k", 0), ("c4_mixed", 0),
           ("c3_bin_64k", 0), ("c4_mixed", 0)]
    dec = ws.frame_decoder()
    used, pols, ms, lats = [], [], [], []
    bufs = {}
    for name, extra in seq:
        if name not in bufs:
            keep = {k: v for k, v in bufs.items() if {k, name} == {"c3_bin_64k", "c4_mixed"}}
            bufs.clear()
            torch.cuda.empty_cache()
            bufs.update(keep)
            bufs[name] = [tools_batch(name), 0]
        (buf, c), k = bufs[name]
        dec.opts = extra
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        r = dec.decode(buf, cap=0, count=True, carry=False)
        b.record()
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
        bufs[name][1] = k + 1
        assert r.nframes == c["decoded_frames"], name
        assert dev_digest(buf) == (c["out_digest"] if (k + 1) % 2 else c["in_digest"]), (name, k)
        assert dec.ctx.last_device_error() == 0
        p = _policy(dec)
        used.append(p[4])
        pols.append(p)
        lats.append(_lat_counters(dec))
    # c3: regular 64 KiB frames (65 550 B with the header): the lattice decoder
    assert pols[1][2] == pols[1][3] == 65550
    assert used[1] == 3 and used[2] == 3
    # the first c4 call after c3 goes to the lattice decoder, which hands the
    # whole batch to the run decoder at once: the run decoder's statistics...
    assert used[3] in (0, 2) and pols[3][2] < pols[3][3]
    # ...after the lattice kernel's prologue handed it over at lattice point 1
    # (its checks, not its segment loop: nothing loaded past the first frames)
    assert lats[3][2] == lats[2][2] + 1 and lats[3][3:] == lats[2][3:], (lats[2], lats[3])
    # ...and the run decoder's time (c4 on the run decoder alone: calls 4, 5;
    # the best of the three c4-after-c3 calls 3, 13, 15 against the best alone)
    assert used[4] in (0, 2) and used[5] in (0, 2)
    assert used[13] in (0, 2) and used[15] in (0, 2)
    assert min(ms[3], ms[13], ms[15]) <= 1.05 * min(ms[4], ms[5]) + 0.02, ms
    # after c4's mixed sizes: the run decoder
    assert used[6] in (0, 2) and used[7] in (0, 2), used
    # c2 after c4: the run decoder, then the lattice
    assert used[8] in (0, 2) and pols[8][2] == pols[8][3] == 264 and used[9] == 3
    assert used[10] in (0, 2)                      # XYWS_OPT_RUNS forces the run decoder
    # c3's first frame is 64 KiB: every lattice call runs 75 KiB segments
    assert lats[2][3] - lats[0][3] == 2 and lats[2][4] == lats[0][4], lats
    # c2's 264-byte frames: 120 KiB segments
    assert lats[9][4] == lats[8][4] + 1, lats


def test_decoder_choice_for_calls_in_flight(ws):
    """The choice for calls enqueued back to back without a synchronisation,
    so that the host's view of the policy words lags behind the device: c3
    three times, then c4 21 times. The lattice decoder's prologue reads the
    previous call's word on the device (HW_DPOL): the first c4 call is the only
    lattice attempt (handed over by its checks at lattice point 1), every later
    c4 call the host still sends to the lattice kernel is handed to the run
    decoder on the policy word before any load of the batch; every c3 call
    runs 75 KiB segments (the first frame's size, this call's). Bytes after
    an odd number of decodes against the reference's output digests."""
    torch.cuda.synchronize()
    c3, k3 = tools_batch("c3_bin_64k")
    c4, k4 = tools_batch("c4_mixed")
    dec = ws.frame_decoder()
    torch.cuda.synchronize()
    dec.decode(c3, cap=0, count=False, carry=False)   # (the stream's past: a lattice call)
    torch.cuda.synchronize()
    l0 = _lat_counters(dec)
    for _ in range(2):
        dec.decode(c3, cap=0, count=False, carry=False)
    for _ in range(21):
        dec.decode(c4, cap=0, count=False, carry=False)
    torch.cuda.synchronize()
    l1 = _lat_counters(dec)
    assert dec.ctx.last_device_error() == 0
    assert dev_digest(c3) == k3["out_digest"]
    assert dev_digest(c4) == k4["out_digest"]
    assert l1[3] - l0[3] == 2 and l1[4] == l0[4], (l0, l1)   # c3: the loops ran, 75 KiB segments
    assert l1[2] - l0[2] == 1, (l0, l1)                      # one lattice attempt on c4
    assert (l1[0] >> 48) & 0x7F in (0, 2) and l1[0] & ((1 << 48) - 1) == 0  # the run decoder, mixed sizes
