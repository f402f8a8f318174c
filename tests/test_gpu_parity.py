"""Parity of the gfx950 path (through the C-ABI) with the reference.

Expected values come from the golden vectors the REAL reference produced
(tests/golden/*.json); per-frame status bits, which the reference does not
compute, come from the oracle (oracle/xyws_oracle.c) run on the same input.
Bar: bit-exact bytes, frames and carries.
"""
import ctypes as C

import numpy as np
import pytest

from conftest import load_golden
import streams

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

OPT_TEST_GIVEUP = 0x100000  # xyws_stream.h: odd runs give up on their successor (finish bridges them)
OPT_STEAL = 0x400000        # work stealing (off by default)
OPT_TEST_STEAL = 0x800000   # every fourth run starts late; pieces of 1 segment and up are taken
OPT_UNMASKED_HINT = 0x2     # include/xyws.h: speculate on server->client framing (wrong for these streams)
OPT_WG512 = 0x40000         # two 512-thread workgroups per CU, 64 KiB segments
OPT_WG256 = 0x8             # four 256-thread workgroups per CU, 16 KiB segments
OPT_NO_LATDEC = 0x800       # the run decoder itself (equal frames would take the lattice decoder)
OPT_LATTICE = 0x400         # the lattice decoder first whatever the previous call found (the bench's decoder)
OPT_BIGSCAN = 0x4000000     # entry scans: one filter pass per segment, whatever the previous call found
MODES = {"fused": {}, "serial": {"serial": True}, "runs1k": {"small_segments": True},
         "lat": {"opts": OPT_LATTICE},
         "bigscan": {"opts": OPT_BIGSCAN | OPT_NO_LATDEC}, "runs1k_bigscan": {"small_segments": True, "opts": OPT_BIGSCAN},
         "wg512": {"opts": OPT_WG512 | OPT_NO_LATDEC}, "wg256": {"opts": OPT_WG256 | OPT_NO_LATDEC},
         "wrong_hint": {"opts": OPT_UNMASKED_HINT | OPT_NO_LATDEC},
         "runs1k_wrong_hint": {"small_segments": True, "opts": OPT_UNMASKED_HINT},
         "giveup": {"opts": OPT_TEST_GIVEUP | OPT_NO_LATDEC},
         "runs1k_giveup": {"small_segments": True, "opts": OPT_TEST_GIVEUP},
         "steal_prod": {"opts": OPT_STEAL | OPT_NO_LATDEC},
         "steal": {"opts": OPT_TEST_STEAL | OPT_NO_LATDEC},
         "runs1k_steal": {"small_segments": True, "opts": OPT_TEST_STEAL},
         "steal_giveup": {"opts": OPT_TEST_STEAL | OPT_TEST_GIVEUP | OPT_NO_LATDEC},
         "runs1k_steal_giveup": {"small_segments": True, "opts": OPT_TEST_STEAL | OPT_TEST_GIVEUP}}


@pytest.fixture(scope="module")
def ws():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from xynet_amd import websocket
    return websocket


def dev_bytes(src: bytes, offset=0, pad=32):
    """src placed at byte `offset` of a guarded device buffer; returns (view, whole)."""
    whole = torch.full((offset + len(src) + pad,), 0xA5, dtype=torch.uint8, device="cuda")
    if src:
        whole[offset:offset + len(src)] = torch.frombuffer(bytearray(src), dtype=torch.uint8).cuda()
    return whole[offset:offset + len(src)], whole


def host(t):
    return t.cpu().numpy().tobytes()


def frames_list(fr, with_status=False):
    out = []
    for f in fr:
        x = [f.frame_off, f.payload_off, f.payload_len, bytes(f.key).hex(), f.flags, f.hdr_len,
             f.status if with_status else f.status & 1]
        out.append(x)
    return out


def carry_list(c):
    return [c.payload_remaining, c.phase, c.frames_total, bytes(c.key).hex(), c.hdr_len,
            bytes(c.hdr[:c.hdr_len]).hex()]


# --------------------------------------------------------------------------- unmask
def test_unmask_golden_vectors(ws, oracle):
    for v in load_golden("unmask.json")["vectors"]:
        rng = streams.SplitMix(v["seed"])
        key = rng.next() & 0xFFFFFFFF
        src = rng.bytes(v["n"])
        for off in (0, 1, 3, 7, 13):
            view, whole = dev_bytes(src, off)
            ret = ws.websocket_mask(view, key, v["phase"])
            assert ret == v["ret"]
            out = host(whole)
            assert out[:off] == b"\xa5" * off and out[off + v["n"]:] == b"\xa5" * 32
            got = out[off:off + v["n"]]
            if "out" in v:
                assert got.hex() == v["out"], (v["n"], v["phase"], off)
            else:
                assert oracle.digest(np.frombuffer(got, np.uint8)) == v["out_digest"]


def test_unmask_is_involution_large(ws):
    n = (64 << 20) + 5
    t = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    ref = t.clone()
    assert ws.websocket_mask(t, 0xDEADBEEF, 3) == n + 3
    assert not torch.equal(t, ref)
    ws.websocket_mask(t, 0xDEADBEEF, 3)
    assert torch.equal(t, ref)


# --------------------------------------------------------------------------- stream
@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("name", streams.EDGE_CASES)
def test_stream_edge_cases(ws, oracle, name, mode):
    g = load_golden("streams.json")["cases"][name]
    src = streams.case_bytes(name)
    for off in (0, 5):
        view, whole = dev_bytes(src, off)
        dec = ws.frame_decoder(**MODES[mode])
        cap = g["nframes"] + 4
        r = dec.decode(view, cap=cap)
        assert r.nframes == g["nframes"]
        out = host(whole)
        assert out[:off] == b"\xa5" * off and out[off + len(src):] == b"\xa5" * 32
        got = np.frombuffer(out[off:off + len(src)], np.uint8)
        assert oracle.digest(got) == g["out_digest"], (name, mode, off)
        if "out" in g:
            assert got.tobytes().hex() == g["out"]
        fr = r.frames()
        assert frames_list(fr) == g["frames"]
        assert carry_list(dec.carry()) == g["carry"]
        # informational status bits: same as the oracle on the same input
        ob = np.frombuffer(src, np.uint8).copy() if src else np.zeros(0, np.uint8)
        ofr, _, _ = oracle.decode_stream(ob)
        assert frames_list(fr, True) == frames_list(ofr, True)


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("name", ["lengths", "tiny_frames", "random_frames_200", "fragments",
                                  "trunc_hdr_9", "len_msb", "random_bytes_3000"])
def test_stream_split_with_carry(ws, name, mode):
    g = load_golden("streams.json")["cases"][name]
    src = streams.case_bytes(name)
    for s in g["splits"]:
        k = s["k"]
        a, wa = dev_bytes(src[:k])
        b, wb = dev_bytes(src[k:])
        dec = ws.frame_decoder(**MODES[mode])
        ra = dec.decode(a, cap=g["nframes"] + 2)
        assert ra.nframes == s["n1"]
        assert carry_list(dec.carry()) == s["carry_mid"], (name, k)
        rb = dec.decode(b, cap=g["nframes"] + 2)
        assert ra.nframes + rb.nframes == g["nframes"]
        assert carry_list(dec.carry()) == g["carry"]
        joined = host(a) + host(b)
        if "out" in g:
            assert joined.hex() == g["out"], (name, k)
        fb = frames_list(rb.frames())
        assert [[x[0] + k, x[1] + k] + x[2:] for x in fb] == g["frames"][s["n1"]:]


@pytest.mark.parametrize("mode", ["fused", "runs1k", "runs1k_giveup", "runs1k_steal", "runs1k_steal_giveup",
                                  "bigscan", "runs1k_bigscan"])
def test_fuzz_random_streams_vs_oracle(ws, oracle, mode):
    """Random frame soups + random cut points, GPU vs oracle."""
    rng = streams.SplitMix(0xF022)
    for it in range(40):
        n = 1 + rng.below(300)
        src = streams.case_bytes(f"random_frames_{n}") if it % 2 else streams.SplitMix(it).bytes(
            rng.below(200000))
        cuts = sorted(set([0, len(src)] + [rng.below(len(src) + 1) for _ in range(rng.below(4))]))
        dec = ws.frame_decoder(**MODES[mode])
        carry = None
        for a, b in zip(cuts[:-1], cuts[1:]):
            piece = src[a:b]
            view, _ = dev_bytes(piece)
            r = dec.decode(view, cap=len(piece) + 2)
            ob = np.frombuffer(piece, np.uint8).copy() if piece else np.zeros(0, np.uint8)
            ofr, carry, on = oracle.decode_stream(ob, carry_in=carry)
            assert r.nframes == on, (it, a, b)
            assert host(view) == ob.tobytes(), (it, a, b)
            assert frames_list(r.frames(), True) == frames_list(ofr, True)
            assert carry_list(dec.carry()) == carry_list(carry)


@pytest.mark.parametrize("mode", ["fused", "bigscan", "runs1k_bigscan"])
@pytest.mark.parametrize("fake", [0, 1, 2])
def test_dense_frames_with_header_like_payloads(ws, oracle, fake, mode):
    """Many small frames (the decoder's dense pass: sub-block chases from
    speculated entries) whose wire payload bytes are themselves chains of
    plausible client headers, so that speculated entries land inside payloads
    and the sequential repair of the dense pass runs (the one-pass entry
    scans: chains of fake headers carried from segment to segment). GPU vs
    oracle: bytes, count, descriptors."""
    rng = streams.SplitMix(0xDE5E + fake)
    out = bytearray()
    while len(out) < (3 << 20):
        plen = 120 + rng.below(400)
        key = rng.bytes(4)
        if fake == 0:
            wire = rng.bytes(plen)
        else:
            # fake 7-byte frames (FIN binary, masked, 1-byte payload) or, for
            # fake == 2, fake 126-form frames that jump within the segment
            unit = (bytes([0x82, 0x81]) + rng.bytes(5)) if fake == 1 else \
                (bytes([0x82, 0xFE, 0x00, 0x40]) + rng.bytes(4) + rng.bytes(64))
            off = rng.below(len(unit))
            wire = (rng.bytes(off) + unit * (plen // len(unit) + 2))[:plen]
        out += streams.header(0x82, plen, key, None) + wire
    src = bytes(out)
    view, _ = dev_bytes(src)
    dec = ws.frame_decoder(**MODES[mode])
    ob = np.frombuffer(src, np.uint8).copy()
    ofr, carry, on = oracle.decode_stream(ob)
    r = dec.decode(view, cap=on + 2)
    assert r.nframes == on
    assert host(view) == ob.tobytes()
    assert frames_list(r.frames(), True) == frames_list(ofr, True)
    assert carry_list(dec.carry()) == carry_list(carry)


@pytest.mark.parametrize("mode", ["fused", "runs1k", "runs1k_giveup", "bigscan", "runs1k_bigscan"])
@pytest.mark.parametrize("kind", ["stride_fakes", "size_changes", "long_lengths", "segment_ends"])
def test_stride_pass_adversarial(ws, oracle, mode, kind):
    """The run decoder's stride pass (lane i parses the header at X + i*F,
    one ballot accepts frames up to the first size change) on streams made
    to mislead it: runs of equal frames whose payloads hold valid headers of
    the same size at every stride offset from the payload start (a stride
    taken from the wrong origin would accept them), runs whose size changes
    every few frames, 126/127-form lengths and 2^31+ lengths in a run,
    and runs crossing segment ends / the batch end. GPU vs oracle: bytes,
    count, descriptors, carry."""
    rng = streams.SplitMix(0x57D1 + len(kind))
    out = bytearray()
    target = 3 << 20 if mode in ("fused", "bigscan") else 200000
    while len(out) < target:
        if kind == "stride_fakes":
            plen = 100 + rng.below(300)
            # the payload: valid headers of frames of exactly `size` bytes at every
            # offset d, d + size, ... from a random d (fake starts on a shifted lattice)
            fake = streams.header(0x82, plen, rng.bytes(4), None)
            size = len(fake) + plen
            d = 1 + rng.below(size - 1)
            body = bytearray(rng.bytes(plen))
            for o in range(d % size, plen - len(fake), size):
                body[o:o + len(fake)] = fake
            for _ in range(1 + rng.below(40)):
                out += streams.header(0x82, plen, rng.bytes(4), None) + bytes(body)
        elif kind == "size_changes":
            plen = rng.below(600)
            for _ in range(1 + rng.below(6)):
                out += streams.frame(rng, 0x82, plen)
        elif kind == "long_lengths":
            for _ in range(1 + rng.below(20)):
                out += streams.frame(rng, 0x81, 126 + rng.below(2))  # 126 form at the 7-bit edge
            out += streams.frame(rng, 0x82, 65536 + rng.below(3))    # 127 form
            if rng.below(8) == 0:
                out += streams.header(0x82, (1 << 31) + rng.below(5), rng.bytes(4), None)  # runs past the end
                break
        else:  # equal frames whose headers straddle 1 KiB and 128 KiB boundaries
            plen = 1024 - 8 - rng.below(24)
            for _ in range(1 + rng.below(200)):
                out += streams.frame(rng, 0x82, plen)
    src = bytes(out)
    for cut in (len(src), len(src) - 5, len(src) - 1000):
        piece = src[:cut]
        view, _ = dev_bytes(piece)
        dec = ws.frame_decoder(**MODES[mode])
        ob = np.frombuffer(piece, np.uint8).copy()
        ofr, carry, on = oracle.decode_stream(ob, cap=len(piece) // 2 + 2)
        r = dec.decode(view, cap=on + 2)
        assert r.nframes == on, (kind, mode, cut)
        assert host(view) == ob.tobytes(), (kind, mode, cut)
        assert frames_list(r.frames(), True) == frames_list(ofr, True)
        assert carry_list(dec.carry()) == carry_list(carry)
        # and without descriptors (the path the bench times; the decoder choice)
        view2, _ = dev_bytes(piece)
        dec2 = ws.frame_decoder(**MODES[mode])
        r2 = dec2.decode(view2, cap=0)
        assert r2.nframes == on and host(view2) == ob.tobytes()


def test_lattice_entry_follows_the_previous_call(ws, oracle):
    """The run decoder's lattice entry (find_entry): after a call whose frames
    were all F bytes long, each run first tries the frame start the lattice
    X0 + kF gives (X0: the batch's first frame). Three calls on one stream:
    equal 264-byte frames twice (sets F = 264; the next calls run in 512-thread
    workgroups; the second takes the lattice entries), then a batch whose first frame is 308 bytes and whose
    payloads hold valid 264-byte headers exactly on the lattice from 0 (every
    run's lattice entry is plausible and wrong: the hand-overs repair it),
    then 520-byte frames (the lattice header has the wrong size: the scan).
    GPU vs oracle: bytes, count, descriptors, carry, for each call."""
    rng = streams.SplitMix(0x1A77)
    target = 8 << 20
    regular = bytearray()
    while len(regular) < target:
        regular += streams.frame(rng, 0x82, 256)
    fakes = bytearray(streams.frame(rng, 0x82, 300))
    while len(fakes) < target:
        fakes += streams.frame(rng, 0x82, 256)
    fake = streams.header(0x82, 256, rng.bytes(4))
    assert len(fake) + 256 == 264
    for k in range(1, len(fakes) // 264):
        o = 264 * k
        if o + len(fake) <= len(fakes):
            fakes[o:o + len(fake)] = fake
    other = bytearray()
    while len(other) < target:
        other += streams.frame(rng, 0x82, 512)
    from xynet_amd import _lib
    stream = torch.cuda.current_stream()
    st = []
    for src in (bytes(regular), bytes(regular), bytes(fakes), bytes(other)):
        # (a new decoder per batch: a fresh carry; the policy words belong to
        # the stream's scratch and stay)
        # (the run decoder itself: equal small frames would take the lattice decoder)
        dec = ws.frame_decoder(opts=_lib.OPT_STATS | _lib.OPT_NO_LATDEC)
        view, _ = dev_bytes(src)
        ob = np.frombuffer(src, np.uint8).copy()
        ofr, carry, on = oracle.decode_stream(ob, cap=len(src) // 8 + 2)
        r = dec.decode(view, cap=on + 2)
        assert r.nframes == on
        assert host(view) == ob.tobytes()
        assert frames_list(r.frames(), True) == frames_list(ofr, True)
        assert carry_list(dec.carry()) == carry_list(carry)
        assert dec.ctx.last_device_error() == 0
        out = (C.c_uint64 * _lib.NSTATS)()
        assert dec.ctx.L.xyws_debug_stats(dec.ctx.h, C.c_void_p(stream.cuda_stream), out) == 0
        st.append(list(out))
    assert st[1][_lib.ST_P_LATTICE] > 0 and st[1][_lib.ST_BAD] == 0  # right: every lattice entry holds
    assert st[2][_lib.ST_P_LATTICE] > 0 and st[2][_lib.ST_BAD] > 0   # plausible and wrong: repaired
    assert st[3][_lib.ST_P_LATTICE] == 0                             # wrong size: scanned


# --------------------------------------------------------------------------- indexed
def test_indexed_matches_golden(ws):
    g = load_golden("streams.json")["cases"]["lengths"]
    src = streams.case_bytes("lengths")
    view, _ = dev_bytes(src, 3)
    r = ws.decode_indexed(view, [f[0] for f in g["frames"]])
    assert host(view).hex() == g.get("out", host(view).hex())
    from conftest import GOLDEN  # noqa: F401
    assert frames_list(r.frames()) == g["frames"]


def test_indexed_overlap_and_tail(ws, oracle):
    src = streams.case_bytes("random_frames_40")
    starts = [0, 5, 5, 100, 2000, len(src) - 3, len(src) + 10]
    view, _ = dev_bytes(src)
    r = ws.decode_indexed(view, starts)
    ob = np.frombuffer(src, np.uint8).copy()
    ofr = oracle.decode_indexed(ob, starts)
    assert host(view) == ob.tobytes()
    assert frames_list(r.frames(), True) == frames_list(ofr, True)


# --------------------------------------------------------------------------- parser mirror
def test_parser_mirror_reference_cases(ws):
    """test/websocket_frame_test.cpp through the device-backed parser."""
    g = load_golden("frame_header.json")
    for c in g["cases"]:
        hb = bytes.fromhex(c["header"])
        p = ws.websocket_frame_header_parser()
        view, _ = dev_bytes(hb)
        assert p.parse(view) == c["ret"]
        f, m, l = p.result()
        assert (int(f), l) == (c["r_flags"], c["r_length"])
        assert ws.websocket_frame_header(c["flags"], c["length"]).span().hex() == c["header"]
    hb = bytes.fromhex(g["cases"][-2]["header"])  # FIN|MASK|PING, 120
    for s in g["splits"]:
        k = s["split"]
        p = ws.websocket_frame_header_parser()
        a, _ = dev_bytes(hb[:k])
        b, _ = dev_bytes(hb[k:])
        assert p.parse(a) == ws.npos
        assert p.parse(b) == s["ret2"]
        assert (int(p.flags()), p.length()) == (s["r_flags"], s["r_length"])


# --------------------------------------------------------------------------- full configs
def tools_batch(name):
    from xynet_amd import _lib
    T = _lib.load_tools()
    c = load_golden("configs.json")["configs"][name]
    buf = torch.empty(c["size"], dtype=torch.uint8, device="cuda")
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    if c["kind"] == "uniform":
        assert T.xyws_tools_fill_uniform(C.c_void_p(buf.data_ptr()), c["nframes"], c["payload"],
                                         c["b0"], c["seed"], s) == 0
    else:
        from xynet_amd._lib import C as _C  # noqa: F401
        tot = C.c_uint64()
        n = T.xyws_tools_mixed_table(c["seed"], c["target"], None, 0, C.byref(tot))
        tab = torch.empty(n * 32, dtype=torch.uint8)
        T.xyws_tools_mixed_table(c["seed"], c["target"], C.c_void_p(tab.data_ptr()), n, C.byref(tot))
        assert tot.value == c["size"]
        dtab = tab.cuda()
        assert T.xyws_tools_fill_mixed(C.c_void_p(buf.data_ptr()), c["size"],
                                       C.c_void_p(dtab.data_ptr()), n, c["seed"], s) == 0
    return buf, c


def dev_digest(buf):
    from xynet_amd import _lib
    T = _lib.load_tools()
    out = torch.zeros(2, dtype=torch.int64, device="cuda")
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert T.xyws_tools_digest(C.c_void_p(buf.data_ptr()), buf.numel(),
                               C.c_void_p(out.data_ptr()), C.c_void_p(out.data_ptr() + 8), s) == 0
    return int(out[0].item()) & ((1 << 64) - 1)


CONFIG_CASES = ([(n, "fused") for n in [
    "t_bin_64k_x64", "t_bin_256_x4096", "t_mixed_8m", "c1_text_4k", "c2_bin_256", "c3_bin_64k",
    "c4_mixed", "c5_shard0", "c5_shard1", "c5_shard4", "c5_shard5", "c5_shard6", "c5_shard7"]] +
    [(n, "lat") for n in ["c1_text_4k", "c2_bin_256", "c3_bin_64k", "c4_mixed", "c5_shard0", "c5_shard1",
                          "c5_shard2", "c5_shard3", "c5_shard4", "c5_shard5", "c5_shard6", "c5_shard7"]] +
    [(n, "bigscan") for n in ["t_bin_64k_x64", "t_bin_256_x4096", "t_mixed_8m", "c1_text_4k", "c2_bin_256", "c3_bin_64k",
                          "c4_mixed", "c5_shard0", "c5_shard3"]] +
    [(n, "runs1k_bigscan") for n in ["t_bin_64k_x64", "t_bin_256_x4096", "t_mixed_8m"]] +
    [(n, "wg512") for n in ["t_mixed_8m", "c1_text_4k", "c2_bin_256", "c3_bin_64k", "c4_mixed"]] +
    [(n, "wg256") for n in ["t_mixed_8m", "c1_text_4k", "c2_bin_256", "c4_mixed"]] +
    [(n, "wrong_hint") for n in ["t_bin_256_x4096", "c4_mixed"]] +
    [(n, "runs1k") for n in ["t_bin_64k_x64", "t_bin_256_x4096", "t_mixed_8m"]] +
    [(n, "giveup") for n in ["t_mixed_8m", "c1_text_4k", "c2_bin_256", "c4_mixed", "c5_shard3"]] +
    [(n, "runs1k_giveup") for n in ["t_bin_256_x4096", "t_mixed_8m"]] +
    [(n, "steal_prod") for n in ["c3_bin_64k", "c4_mixed"]] +
    [(n, "steal") for n in ["t_mixed_8m", "c1_text_4k", "c2_bin_256", "c3_bin_64k", "c4_mixed", "c5_shard2"]] +
    [(n, "runs1k_steal") for n in ["t_bin_256_x4096", "t_mixed_8m", "t_bin_64k_x64"]] +
    [(n, "steal_giveup") for n in ["t_mixed_8m", "c2_bin_256", "c4_mixed"]] +
    [(n, "runs1k_steal_giveup") for n in ["t_mixed_8m"]])


def frames_digest(oracle, r, n):
    return oracle.frames_digest(r.frames_t[: n * 32].cpu().numpy())


@pytest.mark.parametrize("name,mode", CONFIG_CASES)
def test_config_batches(ws, oracle, name, mode):
    """Full bench batches: output bytes, count, carry and the WHOLE descriptor
    table (every frame's offsets, length, key, flags, header length) against
    the reference's (tests/golden/configs.json, from oracle/_ref)."""
    buf, c = tools_batch(name)
    assert dev_digest(buf) == c["in_digest"], "device generator disagrees with the host spec"
    dec = ws.frame_decoder(**MODES[mode])
    n = c["decoded_frames"]
    r = dec.decode(buf, cap=n)
    assert r.nframes == n
    assert dev_digest(buf) == c["out_digest"]
    assert carry_list(dec.carry()) == c["carry"]
    assert frames_list(r.frames()[:4]) == c["first_frames"]
    assert frames_digest(oracle, r, n) == c["frames_digest"]
    assert dec.ctx.last_device_error() == 0
    if mode == "lat":
        # the lattice held over the whole batch (policy word 4 = 3) on the
        # regular configs; c4 is handed to the run decoder at frame 1
        assert (decoder_policy(dec)[4] == 3) == (name != "c4_mixed"), decoder_policy(dec)
    del buf, r
    torch.cuda.empty_cache()


def decoder_policy(dec):
    """The policy words of the last call on the current stream (xyws_debug_policy):
    [epoch, batch bytes, smallest and largest last-frame size, decoder]."""
    out = (C.c_uint64 * 5)()
    stream = torch.cuda.current_stream()
    assert dec.ctx.L.xyws_debug_policy(dec.ctx.h, C.c_void_p(stream.cuda_stream), out) == 0
    return list(out)


@pytest.mark.parametrize("name", ["c1_text_4k", "c2_bin_256", "c3_bin_64k", "c4_mixed", "c5_shard0", "c5_shard7"])
def test_config_batches_bench_path(ws, name):
    """The exact call bench.py times: the full config batch decoded in place
    without descriptors (count on), on the decoder the choice gives a stream
    whose previous calls were this same batch (three calls: an odd count, so
    the payloads end unmasked). Output digest, count and carry against the
    reference's (tests/golden/configs.json); the lattice decoder must be the
    one that finished the regular configs."""
    buf, c = tools_batch(name)
    dec = ws.frame_decoder()
    n = c["decoded_frames"]
    for _ in range(3):
        dec.reset()
        r = dec.decode(buf, cap=0)
        assert r.nframes == n
    assert dev_digest(buf) == c["out_digest"]
    assert carry_list(dec.carry()) == c["carry"]
    assert dec.ctx.last_device_error() == 0
    # the lattice decoder on the regular configs, the run decoder on c4
    assert (decoder_policy(dec)[4] == 3) == (name != "c4_mixed"), decoder_policy(dec)
    del buf, r
    torch.cuda.empty_cache()


@pytest.mark.parametrize("same_ctx", [False, True])
def test_concurrent_decodes_on_two_streams(ws, oracle, same_ctx):
    """Two full-grid decodes at once on two streams (two contexts, or one
    context: per-stream scratch): together they want twice the CUs, so runs
    find successors whose workgroups have not started, give up on them, and
    k_stream_finish bridges the gaps. Both outputs must be the reference's."""
    names = ["c5_shard0", "c5_shard1"]
    batches = [tools_batch(n) for n in names]
    torch.cuda.synchronize()
    streams_ = [torch.cuda.Stream() for _ in names]
    ctx0 = ws.Context(0)
    ctxs = [ctx0, ctx0] if same_ctx else [ctx0, ws.Context(0)]
    decs = [ws.frame_decoder(ctx=c) for c in ctxs]
    results = []
    for rep in range(3):  # odd number of decodes: every payload ends unmasked
        res = []
        for (buf, c), st, dec in zip(batches, streams_, decs):
            with torch.cuda.stream(st):
                dec.reset()
                res.append(dec.decode(buf, cap=c["decoded_frames"]))
        results = res
    torch.cuda.synchronize()
    for (buf, c), r, dec in zip(batches, results, decs):
        assert r.nframes == c["decoded_frames"]
        assert dev_digest(buf) == c["out_digest"]
        assert frames_digest(oracle, r, c["decoded_frames"]) == c["frames_digest"]
        assert carry_list(dec.carry()) == c["carry"]
    for ctx in set(ctxs):
        assert ctx.last_device_error() == 0
    del batches, results
    torch.cuda.empty_cache()


def test_device_error_word_reads_zero_after_clean_decodes(ws):
    dec = ws.frame_decoder()
    src = streams.case_bytes("random_frames_200")
    view, _ = dev_bytes(src)
    dec.decode(view, cap=8)
    assert dec.ctx.last_device_error() == 0
    assert dec.ctx.last_device_error() == 0


@pytest.mark.parametrize("name,small", [("c3_bin_64k", False), ("c4_mixed", False), ("t_mixed_8m", True)])
def test_work_stealing_takes_pieces(ws, oracle, name, small):
    """With late-starting runs (test mode) the runs that finish first take the
    tails of the late runs' ranges: the stats must show accepted splits, and
    bytes, frames and carry must still be the reference's."""
    from xynet_amd import _lib
    buf, c = tools_batch(name)
    dec = ws.frame_decoder(small_segments=small, opts=OPT_TEST_STEAL | _lib.OPT_STATS)
    n = c["decoded_frames"]
    r = dec.decode(buf, cap=n)
    out = (C.c_uint64 * _lib.NSTATS)()
    stream = torch.cuda.current_stream()
    assert dec.ctx.L.xyws_debug_stats(dec.ctx.h, C.c_void_p(stream.cuda_stream), out) == 0
    assert out[_lib.ST_STEAL_ACC] > 0, list(out)
    assert out[_lib.ST_STEAL_SEGS] >= out[_lib.ST_STEAL_ACC]
    assert r.nframes == n
    assert dev_digest(buf) == c["out_digest"]
    assert carry_list(dec.carry()) == c["carry"]
    assert frames_digest(oracle, r, n) == c["frames_digest"]
    assert dec.ctx.last_device_error() == 0
    del buf, r
    torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.parametrize("size", [256 << 10, 1 << 20, 4 << 20, 24 << 20])
def test_dense_first_segment_after_mixed_small_frames(ws, oracle, size):
    """The run decoder's dense0 hint: after a call whose frames were small and
    of mixed sizes, every run's first segment goes to the dense pass at once
    (echo-sized batches: one segment per run). Calls on one stream: mixed
    0-1000 B frames (sets the hint), the same again with descriptors and
    without, then a batch whose payloads are themselves streams of valid
    small frames (the dense pass's speculated entries land on fake headers
    and are checked against the exact chain), then 64 KiB frames (the hint
    off again). GPU vs oracle: bytes, count, descriptors, carry."""
    rng = streams.SplitMix(0xDE45 + size)

    pool, starts = bytearray(), []  # valid small frames, cut at frame starts into payloads
    while len(pool) < (1 << 20):
        starts.append(len(pool))
        pool += streams.frame(rng, 0x81, rng.next() % 120)

    def mixed(fake=False):
        b = bytearray()
        while len(b) < size:
            n = rng.next() % 1001
            if fake:
                o = starts[rng.next() % (len(starts) - 64)]
                inner = bytes(pool[o:o + n])
                b += streams.header(0x82, len(inner), k := rng.bytes(4)) + streams.masked(inner, k)
            else:
                b += streams.frame(rng, 0x81, n)
        return bytes(b[:size - 7])  # (ends inside a frame: the carry)
    big = bytearray()
    while len(big) < size:
        big += streams.frame(rng, 0x82, 65536)
    for src, desc in ((mixed(), True), (mixed(), True), (mixed(), False), (mixed(True), True),
                      (bytes(big[:size]), True)):
        dec = ws.frame_decoder()
        view, _ = dev_bytes(src)
        ob = np.frombuffer(src, np.uint8).copy()
        ofr, carry, on = oracle.decode_stream(ob, cap=len(src) // 6 + 2)
        r = dec.decode(view, cap=on + 2 if desc else 0)
        assert r.nframes == on
        assert host(view) == ob.tobytes()
        if desc:
            assert frames_list(r.frames(), True) == frames_list(ofr, True)
        assert carry_list(dec.carry()) == carry_list(carry)
        assert dec.ctx.last_device_error() == 0
