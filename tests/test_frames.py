"""The callers either side of the decode path, on the device, against the
oracle's restatements (oracle/xyws_oracle.c: oracle_encode_frames,
oracle_classify, oracle_reassemble, oracle_utf8_valid):

  xyws_encode_frames    echo_once's reply build (websocket_echo.cpp:18-27) via
                        detail::websocket_frame_header_builder (:136-175),
                        batched; client-role masking
  xyws_classify_frames  websocket_check_parser_result (websocket.h:81-108)
  xyws_reassemble       FIN=0 chains -> messages, UTF-8 (RFC 3629)

Bar: bit-exact bytes, offsets, verdicts and message records. The oracle's
builder is pinned by the reference's own header bytes (frame_header.json
builds, tests/test_oracle.py); its UTF-8 check by Python's codec (below); the
close policy restates websocket.h:81-108 (no reference test covers it:
parity there is unpinned beyond that restatement).
"""
import codecs
import ctypes as C

import numpy as np
import pytest

import msg_streams
import streams
from oracle.oracle import Frame as OFrame, Verdict as OVerdict

torch = pytest.importorskip("torch")


# --------------------------------------------------------------------------- CPU: oracle pins

@pytest.mark.parametrize("data,complete", [
    ("héllo €𝄞".encode(), True), (b"\xc0\xaf", True), (b"\xed\xa0\x80", True), (b"\xe0\x80\x80", True),
    (b"\xf4\x90\x80\x80", True), (b"\xf4\x8f\xbf\xbf", True), (b"\xe2\x82", True), (b"\xe2\x82", False),
    (b"\xe2\x82\xac\x82", True), (b"", True), (b"\x80", False), (b"abc\xf0\x9f\x98", False),
    (b"\xef\xbf\xbf", True), (b"\xf5\x80\x80\x80", True)])
def test_oracle_utf8_matches_python_codec(oracle, data, complete):
    dec = codecs.getincrementaldecoder("utf-8")()
    try:
        dec.decode(data, final=complete)
        want = True
    except UnicodeDecodeError:
        want = False
    assert oracle.utf8_valid(data, complete) == want


def test_oracle_utf8_random_against_codec(oracle):
    rng = streams.SplitMix(77)
    for _ in range(3000):
        n = rng.below(8)
        b = bytes(rng.below(256) if rng.below(3) else [0x80, 0xC2, 0xE0, 0xED, 0xF0, 0xF4][rng.below(6)]
                  for _ in range(n))
        try:
            b.decode("utf-8")
            want = True
        except UnicodeDecodeError:
            want = False
        assert oracle.utf8_valid(b, True) == want, b.hex()


def test_oracle_reassembly_matches_the_generator(oracle):
    wire, msgs = msg_streams.message_stream(5, nmsg=60)
    host = np.frombuffer(wire, np.uint8).copy()
    frames, _, n = oracle.decode_stream(host)
    out, recs = oracle.reassemble(host, frames, 1)
    complete = [(r.opcode, out[r.out_off:r.out_off + r.length].tobytes()) for r in recs if r.status & 1]
    assert complete == msgs
    for r in recs:
        if r.opcode == 1 and r.status & 1:
            pl = out[r.out_off:r.out_off + r.length].tobytes()
            try:
                pl.decode("utf-8")
                ok = True
            except UnicodeDecodeError:
                ok = False
            assert bool(r.status & 2) == (not ok)


def test_oracle_reference_policy_is_the_bit3_test(oracle):
    """XYWS_POL_REFERENCE restates websocket_check_parser_result in its own
    order (example/include/common/websocket.h:81-108): `flags & WS_OP_CLOSE`
    (bit 3 of the opcode: close, ping, pong, 0xB-0xF) -> 1000, then FIN=0 ->
    1003, unmasked -> 1008, length > max -> 1009."""
    rng = streams.SplitMix(77)
    ops = [0x81, 0x89, 0x8A, 0x8B, 0x88, 0x02, 0x82, 0x8F, 0x80]
    wire = b"".join(streams.frame(rng, b0, 5) for b0 in ops) + streams.frame(rng, 0x81, 3, masked_frame=False) + \
        streams.frame(rng, 0x82, 1001)
    host = np.frombuffer(wire, np.uint8).copy()
    frames, _, n = oracle.decode_stream(host)
    verd, first = oracle.classify(host, frames, 1000, 8)
    want = []
    for f in frames:
        fl = f.flags
        if fl & 0x08:
            want.append(1000)
        elif not fl & 0x10:
            want.append(1003)
        elif not fl & 0x20:
            want.append(1008)
        elif f.payload_len > 1000:
            want.append(1009)
        else:
            want.append(0)
    assert [v.close_code for v in verd] == want
    assert want[:3] == [0, 1000, 1000] and first == 1
    verd0, _ = oracle.classify(host, frames, 1000, 0)
    assert [v.close_code for v in verd0][:4] == [0, 0, 0, 0]  # without the bug: ping, pong, 0xB deliver


def test_oracle_encode_headers_match_reference_builds(oracle):
    from conftest import load_golden
    g = load_golden("frame_header.json")
    for b in g["builds"]:
        src = np.zeros(1, np.uint8)
        f = OFrame()
        f.payload_off, f.payload_len = 0, 0
        if b["length"] > 1 << 20:
            continue  # (the payload would be copied; header bytes are checked in test_oracle)
        f.payload_len = b["length"]
        f.flags = b["flags"]
        src = np.zeros(max(b["length"], 1), np.uint8)
        out, offs, total = oracle.encode_frames(src, [f], b["flags"])
        assert out[:b["size"]].hex() == b["built_nokey"]
        key = bytes.fromhex(b["key"])
        out, offs, total = oracle.encode_frames(src, [f], b["flags"], keys=key)
        want = b["built"] if b["flags"] & 0x20 else b["built_nokey"]
        assert out[:b["size"]].hex() == want


# --------------------------------------------------------------------------- GPU

@pytest.fixture(scope="module")
def ws():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from xynet_amd import websocket
    return websocket


def _decode(ws, oracle, wire):
    """Device decode (frames + unmasked bytes) and the oracle's, which must agree."""
    t = torch.frombuffer(bytearray(wire), dtype=torch.uint8).cuda() if wire else torch.zeros(
        0, dtype=torch.uint8, device="cuda")
    dec = ws.frame_decoder()
    cap = len(wire) // 2 + 2
    r = dec.decode(t, cap=cap)
    n = r.nframes
    host = np.frombuffer(wire, np.uint8).copy() if wire else np.zeros(0, np.uint8)
    ofr, _, on = oracle.decode_stream(host, cap=cap)
    assert n == on
    assert t.cpu().numpy().tobytes() == host.tobytes()
    return t, r.frames_t, n, host, ofr


def _verdicts(raw, n):
    arr = (OVerdict * max(n, 1)).from_buffer_copy(raw.cpu().numpy().tobytes())
    return [arr[i].as_tuple() for i in range(n)]


STREAM_SEEDS = [1, 2, 3]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", STREAM_SEEDS)
@pytest.mark.parametrize("flags,opts,with_keys,cap_frac", [
    (0x11, 0, False, 1.0),    # echo_once: FIN|TEXT, unmasked (server role)
    (0x31, 0, False, 1.0),    # HAS_MASK without keys: the reference class's zero-key form
    (0x20, 1, True, 1.0),     # each frame's own opcode/FIN, ping -> pong, client-role keys
    (0x12, 0, True, 0.6),     # output buffer too small: clipped, total still reported
])
def test_encode_frames_vs_oracle(ws, oracle, seed, flags, opts, with_keys, cap_frac):
    wire, _ = msg_streams.message_stream(seed, nmsg=50)
    wire += b"".join(streams.frame(streams.SplitMix(seed), 0x82, n) for n in (0, 125, 126, 65535, 65536, 70001))
    t, frames_t, n, host, ofr = _decode(ws, oracle, wire)
    rng = streams.SplitMix(seed * 31)
    keys = rng.bytes(4 * n) if with_keys else None
    want, offs, total = oracle.encode_frames(host, ofr, flags, opts, keys)
    cap = int(total * cap_frac)
    want = want[:cap]
    out = torch.full((cap + 48,), 0xA5, dtype=torch.uint8, device="cuda")
    view = out[16:16 + cap]
    dev_keys = torch.frombuffer(bytearray(keys), dtype=torch.uint8).cuda() if keys else None
    dev_offs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
    _, olen = ws.encode_frames(t, frames_t, n, flags, enc_opts=opts, keys=dev_keys, out=view, offsets=dev_offs)
    torch.cuda.synchronize()
    assert int(olen.item()) == total
    assert view.cpu().numpy().tobytes() == want
    assert out[:16].tolist() == [0xA5] * 16 and out[16 + cap:].tolist() == [0xA5] * 32  # nothing outside
    assert dev_offs.cpu().numpy().astype(np.uint64).tolist() == offs.tolist()
    assert ws.context().last_device_error() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("src_shift", [0, 1, 5, 11, 15])
@pytest.mark.parametrize("out_shift", [0, 3, 14])
@pytest.mark.parametrize("short", [False, True])
def test_encode_misaligned_and_short_source(ws, oracle, src_shift, out_shift, short):
    """k_gather's composed chunks at every source/output alignment: the
    decoded batch sits at src_shift in its allocation, the replies at
    out_shift; with `short` the source handed to the encode ends inside the
    last frames' payloads (those bytes read as zero: device error bit 0x100)."""
    rng = streams.SplitMix(src_shift * 7 + out_shift)
    wire = b"".join(streams.frame(rng, 0x82 if i % 3 else 0x81, n)
                    for i, n in enumerate((0, 1, 2, 3, 5, 13, 16, 17, 31, 125, 126, 127, 300, 1000, 4099, 65536)))
    base = torch.zeros(len(wire) + 32, dtype=torch.uint8, device="cuda")
    t = base[src_shift:src_shift + len(wire)]
    t.copy_(torch.frombuffer(bytearray(wire), dtype=torch.uint8))
    dec = ws.frame_decoder()
    r = dec.decode(t, cap=64)
    n = r.nframes
    host = np.frombuffer(wire, np.uint8).copy()
    ofr, _, on = oracle.decode_stream(host, cap=64)
    assert n == on
    slen = len(wire) - (40000 if short else 0)
    src = t[:slen]
    want, offs, total = oracle.encode_frames(host[:slen].copy(), ofr, 0x11)
    out = torch.full((total + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    view = out[out_shift:out_shift + total]
    ws.context().last_device_error()  # (clear)
    _, olen = ws.encode_frames(src, r.frames_t, n, 0x11, out=view)
    torch.cuda.synchronize()
    assert int(olen.item()) == total
    assert view.cpu().numpy().tobytes() == want
    assert out[:out_shift].tolist() == [0xA5] * out_shift
    assert out[out_shift + total:].tolist() == [0xA5] * (64 - out_shift)
    assert ws.context().last_device_error() == (0x100 if short else 0)


@pytest.mark.gpu
def test_encode_selected_by_verdicts_and_device_count(ws, oracle):
    """echo of DATA frames + pongs for pings, frames up to the first close only
    (dev_n = the first closing frame): classify -> encode, all on the device."""
    from xynet_amd import _lib
    rng = streams.SplitMix(99)
    wire, _ = msg_streams.message_stream(9, nmsg=30, orphans=False, interrupted=False)
    wire += msg_streams.close_frame(rng, 1001, b"bye") + streams.frame(rng, 0x81, 40)
    t, frames_t, n, host, ofr = _decode(ws, oracle, wire)
    pol = _lib.POL_FRAGMENTS
    verd, first = ws.classify_frames(t, frames_t, n, 1 << 40, pol)
    overd, ofirst = oracle.classify(host, ofr, 1 << 40, pol)
    assert _verdicts(verd, n) == [v.as_tuple() for v in overd]
    assert int(first.item()) == ofirst < n
    amask = (1 << _lib.ACT_DATA) | (1 << _lib.ACT_PING)
    want, offs, total = oracle.encode_frames(host, ofr[:ofirst], 0x00, _lib.ENC_FRAME_OPCODE, None,
                                             overd[:ofirst], amask)
    out = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
    _, olen = ws.encode_frames(t, frames_t, n, 0x00, dev_n=first, enc_opts=_lib.ENC_FRAME_OPCODE, verdicts=verd,
                               action_mask=amask, out=out)
    assert int(olen.item()) == total
    assert out[:total].cpu().numpy().tobytes() == want


@pytest.mark.gpu
@pytest.mark.parametrize("policy", [0, 1, 2, 5, 7, 8, 9])
@pytest.mark.parametrize("case", ["msgs", "unmasked_mix", "rsv_reserved_ops", "bad_control", "closes"])
def test_classify_vs_oracle(ws, oracle, policy, case):
    rng = streams.SplitMix(123)
    if case == "msgs":
        wire, _ = msg_streams.message_stream(4, unmasked=True)
    elif case == "closes":
        wire = (msg_streams.close_frame(rng) + msg_streams.close_frame(rng, 1000) +
                msg_streams.close_frame(rng, 4000, b"app") + streams.frame(rng, 0x88, 1) +
                streams.frame(rng, 0x89, 3) + streams.frame(rng, 0x8A, 0) + streams.frame(rng, 0x81, 2000))
    else:
        wire = streams.case_bytes(case)
    t, frames_t, n, host, ofr = _decode(ws, oracle, wire)
    for maxp in (1000, 1 << 62):
        verd, first = ws.classify_frames(t, frames_t, n, maxp, policy)
        overd, ofirst = oracle.classify(host, ofr, maxp, policy)
        assert _verdicts(verd, n) == [v.as_tuple() for v in overd]
        assert int(first.item()) & ((1 << 64) - 1) == ofirst


def _messages(raw, cnt):
    from oracle.oracle import Message
    arr = (Message * (len(raw) // 40)).from_buffer_copy(raw.cpu().numpy().tobytes())
    return [arr[i].as_tuple() for i in range(cnt)]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("cap_frac", [1.0, 0.5])
def test_reassemble_vs_oracle(ws, oracle, seed, cap_frac):
    from xynet_amd import _lib
    wire, msgs = msg_streams.message_stream(seed, nmsg=80)
    t, frames_t, n, host, ofr = _decode(ws, oracle, wire)
    total = sum(f.payload_len for f in ofr)
    cap = max(1, int(total * cap_frac))
    oout, orecs = oracle.reassemble(host, ofr, _lib.REASM_UTF8, out_cap=cap)
    out, mt, cnt = ws.reassemble(t, frames_t, n, _lib.REASM_UTF8, out_cap=cap)
    nm = int(cnt.item())
    assert nm == len(orecs)
    assert _messages(mt, nm) == [r.as_tuple() for r in orecs]
    assert out[:cap].cpu().numpy().tobytes() == oout[:cap].tobytes()
    if cap_frac == 1.0:
        got = [(r[5], out[r[2]:r[2] + r[3]].cpu().numpy().tobytes()) for r in _messages(mt, nm) if r[4] & 1]
        assert got == msgs  # every complete message, as the generator wrote it
    ws.context().last_device_error()  # (clears bit 0x200: this stream may end in orphan continuations)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [3, 8])
def test_reassemble_small_msg_cap_and_trailing_orphans(ws, oracle, seed):
    """msg_cap below the message count: every stored record is the oracle's
    (the last one ends at the next message's start, not at the batch end);
    continuations after the last message set bit 0x200 of the error word."""
    from xynet_amd import _lib
    rng = streams.SplitMix(seed)
    wire, _ = msg_streams.message_stream(seed, nmsg=60)
    wire += msg_streams._frame(rng, 0x82, rng.bytes(10))  # a whole message (closes any open one)...
    wire += msg_streams._frame(rng, 0x80, rng.bytes(30))  # ...then an orphan continuation, no message after it
    t, frames_t, n, host, ofr = _decode(ws, oracle, wire)
    oout, orecs = oracle.reassemble(host, ofr, _lib.REASM_UTF8)
    for cap in (1, len(orecs) // 2, len(orecs) - 1):
        ws.context().last_device_error()  # (clear)
        out, mt, cnt = ws.reassemble(t, frames_t, n, _lib.REASM_UTF8, msg_cap=cap)
        assert int(cnt.item()) == len(orecs)
        assert _messages(mt, cap) == [r.as_tuple() for r in orecs[:cap]]
        assert ws.context().last_device_error() == 0x200


@pytest.mark.gpu
def test_reassemble_text_utf8_fragments_split_inside_sequences(ws, oracle):
    """Fragments cut inside multi-byte sequences: valid after gathering."""
    from xynet_amd import _lib
    rng = streams.SplitMix(7)
    text = ("€𝄞 日本語 ✓ " * 50).encode()
    wire = b""
    for k in range(1, 8):
        parts = msg_streams.split_parts(rng, text, k)
        for i, p in enumerate(parts):
            wire += msg_streams._frame(rng, (1 if i == 0 else 0) | (0x80 if i == k - 1 else 0), p)
    wire += msg_streams._frame(rng, 0x81, text.rstrip()[:-1])  # cut inside the last sequence: invalid
    t, frames_t, n, host, ofr = _decode(ws, oracle, wire)
    out, mt, cnt = ws.reassemble(t, frames_t, n, _lib.REASM_UTF8)
    recs = _messages(mt, int(cnt.item()))
    assert [r[4] & 3 for r in recs] == [1] * 7 + [3]


@pytest.mark.gpu
def test_reassemble_utf8_probe_window(ws, oracle):
    """k_utf8's probe pass (a text message's first 16 bytes, and the 3 bytes
    either side its rules read) and the streaming pass's skip of the messages
    it marks: an invalid byte, an overlong or surrogate lead, an out-of-range
    code point, a cut sequence, or a VALID 2/3/4-byte sequence, at every
    position 0..23 of text messages of 1..40 bytes, some fragmented, some
    crossing a 64 KiB UTF-8 tile boundary (records and bytes against the
    oracle's)."""
    from xynet_amd import _lib
    rng = streams.SplitMix(0x0F)
    wire = msg_streams._frame(rng, 0x82, bytes(65536 - 2000))  # (the text messages cross the first tile end)
    seqs = [b"\x80", b"\xc0\xaf", b"\xe0\x80\x80", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\xff", b"\xe2\x82",
            "\u00e9".encode(), "\u20ac".encode(), "\U0001d11e".encode()]
    k = 0
    for length in (1, 3, 15, 16, 17, 18, 19, 20, 24, 40):
        for pos in range(min(length, 24)):
            seq = seqs[k % len(seqs)]
            k += 1
            body = (b"x" * pos + seq + b"y" * length)[:length]
            if k % 5 == 0 and length > 2:  # two fragments, cut inside the probe window
                cut = rng.below(length)
                wire += msg_streams._frame(rng, 0x01, body[:cut]) + msg_streams._frame(rng, 0x80, body[cut:])
            else:
                wire += msg_streams._frame(rng, 0x81, body)
    t, frames_t, n, host, ofr = _decode(ws, oracle, wire)
    oout, orecs = oracle.reassemble(host, ofr, _lib.REASM_UTF8)
    out, mt, cnt = ws.reassemble(t, frames_t, n, _lib.REASM_UTF8)
    nm = int(cnt.item())
    assert nm == len(orecs)
    got, want = _messages(mt, nm), [r.as_tuple() for r in orecs]
    assert got == want
    assert sum(1 for r in want if r[4] & 2) > 100 and sum(1 for r in want if r[5] == 1 and not r[4] & 2) > 30
    assert out[:len(oout)].cpu().numpy().tobytes() == oout.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c2_bin_256", "c3_bin_64k"])
def test_echo_round_trip_full_config(ws, name):
    """At a bench configuration: decode the batch, build client-role replies
    with fresh keys, decode those, gather both payload sets: identical bytes
    (encode -> decode is the identity on payloads), byte counts add up."""
    from test_gpu_parity import tools_batch
    buf, c = tools_batch(name)
    n = c["decoded_frames"]
    dec = ws.frame_decoder()
    r = dec.decode(buf, cap=n)
    assert r.nframes == n
    keys = torch.randint(0, 256, (4 * n,), dtype=torch.uint8, device="cuda")
    total_payload = int(r.frames_t[: n * 32].view(torch.int64).view(n, 4)[:, 2].sum().item())
    out = torch.empty(buf.numel() + 16 * n + 64, dtype=torch.uint8, device="cuda")
    _, olen = ws.encode_frames(buf, r.frames_t, n, 0x22, keys=keys, out=out)
    rep_len = int(olen.item())
    assert rep_len <= out.numel()
    reply = out[:rep_len]
    dec2 = ws.frame_decoder()
    r2 = dec2.decode(reply, cap=n)
    assert r2.nframes == n
    g1, m1, c1 = ws.reassemble(buf, r.frames_t, n, 0, out_cap=total_payload)
    g2, m2, c2 = ws.reassemble(reply, r2.frames_t, n, 0, out_cap=total_payload)
    assert int(c1.item()) == int(c2.item()) == n
    assert torch.equal(g1, g2)
    assert ws.context().last_device_error() == 0
    del buf, out, reply, g1, g2
    torch.cuda.empty_cache()
