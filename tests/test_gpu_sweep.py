"""Parity of the sweep decoder (k_stream_sweep: the path of every
xyws_decode_stream call that asks for no descriptors, the headline's) with the
reference, through the C-ABI.

Expected values come from the golden vectors the REAL reference produced
(tests/golden/*.json) and from the oracle (oracle/xyws_oracle.c) on the same
input. Bar: bit-exact bytes, frame counts and carries. The test modes force
the sweep's rare paths on small inputs: 1 KiB segments (many segments, entering
states handed over between them, frames spanning many segments, headers cut by
segment ends), segments that pretend to find no frame start or speculate one
byte late (look-back fix-ups, deferred segments, the finisher's repair walk),
and the wrong framing hint (every speculation fails).
"""
import ctypes as C

import numpy as np
import pytest

from conftest import load_golden
import streams
from test_gpu_parity import carry_list, dev_bytes, dev_digest, host, tools_batch

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

OPT_UNMASKED_HINT = 0x2     # include/xyws.h: speculate on server->client framing (wrong for these streams)
OPT_SWEEP = 0x1000000       # xyws_stream.h: the sweep decoder instead of the run decoder
OPT_TEST_SPEC = 0x2000000   # xyws_stream.h: forced mis-speculation (segments 1, 4, ...: none; 2, 5, ...: late)
MODES = {"sweep": {"opts": OPT_SWEEP}, "sweep1k": {"small_segments": True, "opts": OPT_SWEEP},
         "sweep_spec": {"opts": OPT_SWEEP | OPT_TEST_SPEC},
         "sweep1k_spec": {"small_segments": True, "opts": OPT_SWEEP | OPT_TEST_SPEC},
         "sweep_wrong_hint": {"opts": OPT_SWEEP | OPT_UNMASKED_HINT},
         "sweep1k_wrong_hint": {"small_segments": True, "opts": OPT_SWEEP | OPT_UNMASKED_HINT},
         "sweep1k_spec_wrong_hint": {"small_segments": True, "opts": OPT_SWEEP | OPT_TEST_SPEC | OPT_UNMASKED_HINT}}


@pytest.fixture(scope="module")
def ws():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from xynet_amd import websocket
    return websocket


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("name", streams.EDGE_CASES)
def test_sweep_edge_cases(ws, oracle, name, mode):
    g = load_golden("streams.json")["cases"][name]
    src = streams.case_bytes(name)
    for off in (0, 5, 13):
        view, whole = dev_bytes(src, off)
        dec = ws.frame_decoder(**MODES[mode])
        r = dec.decode(view)
        assert r.nframes == g["nframes"], (name, mode, off)
        out = host(whole)
        assert out[:off] == b"\xa5" * off and out[off + len(src):] == b"\xa5" * 32
        got = np.frombuffer(out[off:off + len(src)], np.uint8)
        assert oracle.digest(got) == g["out_digest"], (name, mode, off)
        if "out" in g:
            assert got.tobytes().hex() == g["out"]
        assert carry_list(dec.carry()) == g["carry"], (name, mode, off)
        assert dec.ctx.last_device_error() == 0


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("name", ["lengths", "tiny_frames", "random_frames_200", "fragments",
                                  "trunc_hdr_9", "len_msb", "random_bytes_3000"])
def test_sweep_split_with_carry(ws, name, mode):
    g = load_golden("streams.json")["cases"][name]
    src = streams.case_bytes(name)
    for s in g["splits"]:
        k = s["k"]
        a, _ = dev_bytes(src[:k])
        b, _ = dev_bytes(src[k:])
        dec = ws.frame_decoder(**MODES[mode])
        ra = dec.decode(a)
        assert ra.nframes == s["n1"], (name, k)
        assert carry_list(dec.carry()) == s["carry_mid"], (name, k)
        rb = dec.decode(b)
        assert ra.nframes + rb.nframes == g["nframes"]
        assert carry_list(dec.carry()) == g["carry"]
        if "out" in g:
            assert (host(a) + host(b)).hex() == g["out"], (name, k)


@pytest.mark.parametrize("mode", list(MODES))
def test_sweep_fuzz_vs_oracle(ws, oracle, mode):
    """Random frame soups and random bytes cut at random points, GPU vs oracle."""
    rng = streams.SplitMix(0x5EE9)
    for it in range(30):
        n = 1 + rng.below(400)
        src = streams.case_bytes(f"random_frames_{n}") if it % 2 else streams.SplitMix(it + 77).bytes(
            rng.below(300000))
        cuts = sorted(set([0, len(src)] + [rng.below(len(src) + 1) for _ in range(rng.below(4))]))
        dec = ws.frame_decoder(**MODES[mode])
        carry = None
        for a, b in zip(cuts[:-1], cuts[1:]):
            piece = src[a:b]
            view, _ = dev_bytes(piece, a & 15)
            r = dec.decode(view)
            ob = np.frombuffer(piece, np.uint8).copy() if piece else np.zeros(0, np.uint8)
            _, carry, on = oracle.decode_stream(ob, carry_in=carry)
            assert r.nframes == on, (it, a, b)
            assert host(view) == ob.tobytes(), (it, a, b)
            assert carry_list(dec.carry()) == carry_list(carry), (it, a, b)
        assert dec.ctx.last_device_error() == 0


def big_frames_stream(seed, sizes, total):
    """Masked frames with payload sizes drawn from `sizes` until `total` bytes."""
    rng = streams.SplitMix(seed)
    out = bytearray()
    while len(out) < total:
        plen = sizes[rng.below(len(sizes))]
        b0 = 0x82 if rng.below(4) else 0x02
        out += streams.header(b0, plen, rng.bytes(4), None) + rng.bytes(plen)
    return bytes(out)


@pytest.mark.parametrize("mode", ["sweep", "sweep_spec", "sweep1k", "sweep1k_spec"])
@pytest.mark.parametrize("kind", ["huge", "cut_headers", "mixed"])
def test_sweep_segment_boundaries(ws, oracle, mode, kind):
    """Frames far larger than a segment (segments that publish no state and
    look back past several), and frames whose headers straddle segment ends at
    every offset (the pad bytes after a segment)."""
    if kind == "huge":
        src = big_frames_stream(0x1A, [300000, 700000, 5, 131000, 131072, 131073], 6 << 20)
    elif kind == "cut_headers":
        # payload sizes that walk header starts across every offset of a 1 KiB
        # and a 128 KiB segment end
        sizes = [131072 - 14 - d for d in range(0, 20)] + [1024 - 8 - d for d in range(0, 16)] + \
                [1024 - 14 - d for d in range(0, 16)]
        src = big_frames_stream(0x2B, sizes, 5 << 20)
    else:
        src = big_frames_stream(0x3C, [0, 1, 125, 126, 127, 65535, 65536, 65537, 1000, 4096], 4 << 20)
    view, _ = dev_bytes(src, 3)
    dec = ws.frame_decoder(**MODES[mode])
    ob = np.frombuffer(src, np.uint8).copy()
    _, carry, on = oracle.decode_stream(ob)
    r = dec.decode(view)
    assert r.nframes == on
    assert host(view) == ob.tobytes()
    assert carry_list(dec.carry()) == carry_list(carry)
    assert dec.ctx.last_device_error() == 0


@pytest.mark.parametrize("fake", [0, 1, 2])
@pytest.mark.parametrize("mode", ["sweep", "sweep_spec"])
def test_sweep_dense_header_like_payloads(ws, oracle, fake, mode):
    """Many small frames whose payloads are chains of plausible client
    headers (false speculated entries inside payloads)."""
    rng = streams.SplitMix(0xDE5E + fake)
    out = bytearray()
    while len(out) < (3 << 20):
        plen = 120 + rng.below(400)
        key = rng.bytes(4)
        if fake == 0:
            wire = rng.bytes(plen)
        else:
            unit = (bytes([0x82, 0x81]) + rng.bytes(5)) if fake == 1 else \
                (bytes([0x82, 0xFE, 0x00, 0x40]) + rng.bytes(4) + rng.bytes(64))
            off = rng.below(len(unit))
            wire = (rng.bytes(off) + unit * (plen // len(unit) + 2))[:plen]
        out += streams.header(0x82, plen, key, None) + wire
    src = bytes(out)
    view, _ = dev_bytes(src)
    dec = ws.frame_decoder(**MODES[mode])
    ob = np.frombuffer(src, np.uint8).copy()
    _, carry, on = oracle.decode_stream(ob)
    r = dec.decode(view)
    assert r.nframes == on
    assert host(view) == ob.tobytes()
    assert carry_list(dec.carry()) == carry_list(carry)


SWEEP_CONFIGS = ([(n, "sweep") for n in [
    "t_bin_64k_x64", "t_bin_256_x4096", "t_mixed_8m", "c1_text_4k", "c2_bin_256", "c3_bin_64k",
    "c4_mixed", "c5_shard0", "c5_shard1", "c5_shard2", "c5_shard3", "c5_shard4", "c5_shard5", "c5_shard6",
    "c5_shard7"]] +
    [(n, "sweep_spec") for n in ["t_mixed_8m", "c2_bin_256", "c3_bin_64k", "c4_mixed"]] +
    [(n, "sweep_wrong_hint") for n in ["t_bin_256_x4096", "t_mixed_8m"]] +
    [(n, "sweep1k") for n in ["t_bin_64k_x64", "t_bin_256_x4096", "t_mixed_8m"]] +
    [(n, "sweep1k_spec") for n in ["t_bin_256_x4096", "t_mixed_8m"]])


@pytest.mark.parametrize("name,mode", SWEEP_CONFIGS)
def test_sweep_config_batches(ws, name, mode):
    """Full bench batches: output bytes, count and carry against the
    reference's (tests/golden/configs.json, from oracle/_ref)."""
    buf, c = tools_batch(name)
    assert dev_digest(buf) == c["in_digest"], "device generator disagrees with the host spec"
    dec = ws.frame_decoder(**MODES[mode])
    r = dec.decode(buf)
    assert r.nframes == c["decoded_frames"]
    assert dev_digest(buf) == c["out_digest"]
    assert carry_list(dec.carry()) == c["carry"]
    # a second decode re-masks the batch: the input again (XOR is an involution)
    dec.reset()
    r = dec.decode(buf)
    assert r.nframes == c["decoded_frames"]
    assert dev_digest(buf) == c["in_digest"]
    assert dec.ctx.last_device_error() == 0
    del buf, r
    torch.cuda.empty_cache()


def test_sweep_matches_run_decoder(ws):
    """The two decoders on the same batch: the same bytes and count."""
    buf, c = tools_batch("t_mixed_8m")
    ref = buf.clone()
    a = ws.frame_decoder(opts=OPT_SWEEP).decode(buf)
    b = ws.frame_decoder().decode(ref)
    assert a.nframes == b.nframes == c["decoded_frames"]
    assert torch.equal(buf, ref)


@pytest.mark.parametrize("same_ctx", [False, True])
def test_sweep_concurrent_decodes(ws, same_ctx):
    """Two full-grid sweeps at once on two streams (two contexts, or one
    context: per-stream scratch): each claims its own segments; both outputs
    must be the reference's."""
    names = ["c5_shard0", "c5_shard1"]
    batches = [tools_batch(n) for n in names]
    torch.cuda.synchronize()
    streams_ = [torch.cuda.Stream() for _ in names]
    ctx0 = ws.Context(0)
    ctxs = [ctx0, ctx0] if same_ctx else [ctx0, ws.Context(0)]
    decs = [ws.frame_decoder(ctx=c, opts=OPT_SWEEP) for c in ctxs]
    results = []
    for rep in range(3):
        res = []
        for (buf, c), st, dec in zip(batches, streams_, decs):
            with torch.cuda.stream(st):
                dec.reset()
                res.append(dec.decode(buf))
        results = res
    torch.cuda.synchronize()
    for (buf, c), r, dec in zip(batches, results, decs):
        assert r.nframes == c["decoded_frames"]
        assert dev_digest(buf) == c["out_digest"]
        assert carry_list(dec.carry()) == c["carry"]
    for ctx in set(ctxs):
        assert ctx.last_device_error() == 0
    del batches, results
    torch.cuda.empty_cache()


def test_sweep_stats_show_no_repairs_on_c3(ws):
    """On the headline batch every segment's speculation holds: no segment
    whose final exit differs from its publication, no repair step."""
    from xynet_amd import _lib
    buf, c = tools_batch("c3_bin_64k")
    dec = ws.frame_decoder(opts=_lib.OPT_STATS | OPT_SWEEP)
    r = dec.decode(buf)
    out = (C.c_uint64 * _lib.NSTATS)()
    stream = torch.cuda.current_stream()
    assert dec.ctx.L.xyws_debug_stats(dec.ctx.h, C.c_void_p(stream.cuda_stream), out) == 0
    assert r.nframes == c["decoded_frames"]
    # (ST_SEGS also counts dense passes: >= the segment count)
    assert out[_lib.ST_SEGS] >= (c["size"] + (128 << 10) - 1) // (128 << 10), list(out)
    assert out[_lib.ST_BAD] == 0 and out[_lib.ST_REPAIR] == 0, list(out)
    # exact-mode segments (entering state first): segment 0, and at most a
    # workgroup's first segment (no stride reference yet) whose quick scan missed
    assert out[_lib.ST_SW_DEFER] <= 1024, list(out)
    del buf, r
    torch.cuda.empty_cache()


def _policy(dec):
    out = (C.c_uint64 * 5)()
    stream = torch.cuda.current_stream()
    assert dec.ctx.L.xyws_debug_policy(dec.ctx.h, C.c_void_p(stream.cuda_stream), out) == 0
    return list(out)


def test_decoder_choice_follows_the_frames(ws):
    """The decoder choice (stream_decode_fused): the lattice decoder first when
    the previous call on the stream found frames of one size (>= 128 B, policy
    word 4 = 3), the run decoder otherwise (0, or 2 in 512-thread workgroups
    after regular frames under 2 KiB). An irregular batch after regular ones
    goes to the lattice decoder, which hands it to the run decoder at its first
    size change: its time stays that of the run decoder alone (the decoder-
    choice cliff of round 3 was 7x: the sweep decoder scanning every segment).
    Every call is checked against the reference's digests, whichever decoder
    ran."""
    from xynet_amd import _lib
    seq = [("c3_bin_64k", 0), ("c3_bin_64k", 0), ("c3_bin_64k", 0), ("c4_mixed", 0), ("c4_mixed", 0),
           ("c4_mixed", 0), ("c2_bin_256", 0), ("c2_bin_256", 0), ("c3_bin_64k", _lib.OPT_RUNS)]
    dec = ws.frame_decoder()
    used, pols, ms = [], [], []
    bufs = {}
    for name, extra in seq:
        if name not in bufs:
            bufs.clear()
            torch.cuda.empty_cache()
            bufs[name] = [tools_batch(name), 0]
        (buf, c), k = bufs[name]
        dec.opts = extra
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
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
    # c3: regular 64 KiB frames (65 550 B with the header): the lattice decoder
    assert pols[1][2] == pols[1][3] == 65550
    assert used[1] == 3 and used[2] == 3
    # the first c4 call after c3 goes to the lattice decoder and is handed to
    # the run decoder at its second frame: the run decoder's statistics...
    assert used[3] in (0, 2) and pols[3][2] < pols[3][3]
    # ...and the run decoder's time (c4 alone on the run decoder: calls 4, 5)
    assert ms[3] <= 1.25 * min(ms[4], ms[5]) + 0.05, ms
    assert used[4] in (0, 2) and used[5] in (0, 2)
    # after c4's irregular frames: the run decoder for c2, then the lattice
    assert used[6] in (0, 2) and pols[6][2] == pols[6][3] == 264 and used[7] == 3
    assert used[8] in (0, 2)                      # XYWS_OPT_RUNS forces the run decoder
