"""The CPU oracle (oracle/xyws_oracle.c) against the golden vectors produced
from the REAL reference headers (tests/golden/gen_golden.py) — this pins the
restatement before any GPU result is compared with it."""
import numpy as np
import pytest

from conftest import load_golden
import streams

NPOS = (1 << 64) - 1


def test_reference_frame_header_cases(oracle):
    """test/websocket_frame_test.cpp:10-65 — build -> parse round trip."""
    g = load_golden("frame_header.json")
    for c in g["cases"]:
        hb = oracle.header_build(c["flags"], None, c["length"])
        assert hb.hex() == c["header"]
        p = oracle.parser()
        assert p.parse(hb) == c["ret"] == len(hb)
        f, m, l = p.result()
        assert (f, m, l) == (c["r_flags"], c["r_mask"], c["r_length"])
        assert f == c["flags"] and l == c["length"]


def test_reference_split_parse(oracle):
    """test/websocket_frame_test.cpp:67-89 — header fed in two spans at every split."""
    g = load_golden("frame_header.json")
    hb = oracle.header_build(0x10 | 0x20 | 0x09, None, 120)
    for s in g["splits"]:
        p = oracle.parser()
        k = s["split"]
        assert p.parse(hb[:k]) == s["ret1"] == NPOS
        assert p.parse(hb[k:]) == s["ret2"]
        f, _, l = p.result()
        assert (f, l) == (s["r_flags"], s["r_length"])


def test_builder_and_sizes(oracle):
    g = load_golden("frame_header.json")
    assert g["max_header_size"] == 14
    for b in g["builds"]:
        key = bytes.fromhex(b["key"])
        assert oracle.header_build(b["flags"], key, b["length"]).hex() == b["built"]
        assert oracle.header_build(b["flags"], None, b["length"]).hex() == b["built_nokey"]
        # masked-ctor quirk (websocket_frame_header.h:191-202): key never reaches the header
        assert b["ctor_masked"] == b["built_nokey"]
        assert oracle.calc_frame_header_size(b["flags"], b["length"]) == b["size"]


def test_parse_corpus(oracle):
    for c in load_golden("parse_corpus.json")["corpus"]:
        hb = bytes.fromhex(c["bytes"])
        p = oracle.parser()
        assert p.parse(hb) == c["ret"], c["bytes"]
        assert p.result() == (c["flags"], c["mask"], c["length"]), c["bytes"]
        if hb:
            assert p.parse(hb) == c["again"]
        q = oracle.parser()
        assert [q.parse(hb[i:i + 1]) for i in range(len(hb))] == c["feed"], c["bytes"]
        assert q.result() == (c["feed_flags"], c["feed_mask"], c["feed_length"])


def test_rfc6455_hello(oracle):
    """RFC 6455 §5.7 single-frame masked text "Hello"."""
    buf = np.frombuffer(bytes.fromhex("818537fa213d7f9f4d5158"), np.uint8).copy()
    frames, carry, n = oracle.decode_stream(buf)
    assert n == 1 and bytes(buf[6:]) == b"Hello"
    f = frames[0]
    assert (f.frame_off, f.payload_off, f.payload_len, bytes(f.key), f.flags, f.hdr_len) == \
        (0, 6, 5, bytes.fromhex("37fa213d"), 0x31, 6)


def test_unmask_vectors(oracle):
    for v in load_golden("unmask.json")["vectors"]:
        rng = streams.SplitMix(v["seed"])
        key = rng.next() & 0xFFFFFFFF
        assert key == v["key"]
        data = np.frombuffer(rng.bytes(v["n"]), np.uint8).copy() if v["n"] else np.zeros(0, np.uint8)
        assert oracle.mask(data, key, v["phase"]) == v["ret"]
        if "out" in v:
            assert data.tobytes().hex() == v["out"]
        else:
            assert oracle.digest(data) == v["out_digest"]


def _frames(fr):
    return [[f.frame_off, f.payload_off, f.payload_len, bytes(f.key).hex(), f.flags, f.hdr_len,
             f.status & 1] for f in fr]


def _carry(c):
    return [c.payload_remaining, c.phase, c.frames_total, bytes(c.key).hex(), c.hdr_len,
            bytes(c.hdr[:c.hdr_len]).hex()]


@pytest.mark.parametrize("name", streams.EDGE_CASES)
def test_stream_cases(oracle, name):
    g = load_golden("streams.json")["cases"][name]
    src = streams.case_bytes(name)
    assert len(src) == g["size"]
    buf = np.frombuffer(src, np.uint8).copy() if src else np.zeros(0, np.uint8)
    assert oracle.digest(buf) == g["in_digest"]
    frames, carry, n = oracle.decode_stream(buf)
    assert n == g["nframes"]
    assert _frames(frames) == g["frames"]
    assert _carry(carry) == g["carry"]
    assert oracle.digest(buf) == g["out_digest"]
    if "out" in g:
        assert buf.tobytes().hex() == g["out"]
    for s in g["splits"]:
        k = s["k"]
        a = np.frombuffer(src[:k], np.uint8).copy() if k else np.zeros(0, np.uint8)
        b = np.frombuffer(src[k:], np.uint8).copy() if k < len(src) else np.zeros(0, np.uint8)
        fa, ca, na = oracle.decode_stream(a)
        assert na == s["n1"] and _carry(ca) == s["carry_mid"], (name, k)
        fb, cb, nb = oracle.decode_stream(b, carry_in=ca)
        assert oracle.digest(np.concatenate([a, b])) == g["out_digest"], (name, k)
        assert na + nb == n
        # frames of the second half are the whole-stream frames, shifted by k
        assert [[x[0] + k, x[1] + k] + x[2:] for x in _frames(fb)] == g["frames"][na:], (name, k)


@pytest.mark.parametrize("name", ["t_bin_64k_x64", "t_bin_256_x4096", "t_mixed_8m",
                                  "c1_text_4k", "c2_bin_256"])
def test_config_digests(oracle, name):
    c = load_golden("configs.json")["configs"][name]
    if c["kind"] == "uniform":
        buf = oracle.fill_uniform(c["nframes"], c["payload"], c["b0"], c["seed"])
    else:
        tab, n, total = oracle.mixed_table(c["seed"], c["target"])
        assert n == c["nframes"]
        buf = oracle.fill_mixed(tab, n, total, c["seed"])
    assert buf.size == c["size"]
    assert oracle.digest(buf) == c["in_digest"]
    raw, carry, n = oracle.decode_stream_raw(buf, c["decoded_frames"])
    assert n == c["decoded_frames"]
    assert oracle.digest(buf) == c["out_digest"]
    assert _carry(carry) == c["carry"]
    from oracle.oracle import Frame
    assert _frames(list((Frame * 4).from_buffer_copy(raw[:128].tobytes()))) == c["first_frames"]
    # the whole descriptor table, against the reference's
    assert oracle.frames_digest(raw) == c["frames_digest"]


def test_indexed_matches_stream(oracle):
    """Indexed decode at the stream's own boundaries == stream decode."""
    src = streams.case_bytes("lengths")
    a = np.frombuffer(src, np.uint8).copy()
    fr, _, n = oracle.decode_stream(a)
    b = np.frombuffer(src, np.uint8).copy()
    fi = oracle.decode_indexed(b, [f.frame_off for f in fr])
    assert (a == b).all()
    assert _frames(fi) == _frames(fr)
