"""Device paths the round-1 parity suite did not reach (gpu):

* the reference's parser corpus (tests/golden/parse_corpus.json, written by
  the real websocket_frame_header_parser, websocket_frame_header.h:226-385)
  through the DEVICE-backed parser (xyws_parser_*): whole-header parse,
  re-feed after completion, and byte-at-a-time feeding with the npos protocol;
* server->client (unmasked) streams decoded with XYWS_OPT_UNMASKED_HINT, in the
  production geometry and in 1 KiB-segment runs (every run boundary
  speculated on unmasked headers), and client streams decoded with the WRONG
  hint (speculation fails everywhere; the repair must keep them exact);
(the two-workgroups-per-CU geometry, XYWS_OPT_WG512, and the unmasked hint on
client streams run as modes of test_gpu_parity's edge-case, split and
configuration tests.)
Bar: bit-exact bytes, frames, carries (oracle = the pinned restatement where
no golden covers the input; parity for those inputs is pinned through it).
"""
import numpy as np
import pytest

from conftest import load_golden
import streams
from test_gpu_parity import carry_list, dev_bytes, frames_list, host, torch

pytestmark = pytest.mark.gpu

OPT_UNMASKED_HINT = 0x2   # include/xyws.h


@pytest.fixture(scope="module")
def ws():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from xynet_amd import websocket
    return websocket


def test_parse_corpus_on_device(ws):
    for c in load_golden("parse_corpus.json")["corpus"]:
        hb = bytes.fromhex(c["bytes"])
        p = ws.websocket_frame_header_parser()
        assert p.parse(hb) == c["ret"], c["bytes"]
        f, m, ln = p.result()
        assert (int(f), m, ln) == (c["flags"], c["mask"], c["length"]), c["bytes"]
        if hb:
            assert p.parse(hb) == c["again"], c["bytes"]
        q = ws.websocket_frame_header_parser()
        assert [q.parse(hb[i:i + 1]) for i in range(len(hb))] == c["feed"], c["bytes"]
        f, m, ln = q.result()
        assert (int(f), m, ln) == (c["feed_flags"], c["feed_mask"], c["feed_length"]), c["bytes"]
        # reset() starts a new header (websocket_frame_header.h:378-384)
        q.reset()
        assert q.parse(hb) == c["ret"], c["bytes"]


def server_stream(seed, nbytes, small=True):
    """Back-to-back server->client frames (MASK = 0), FIN binary/text/continuation
    and pings, payload sizes from 0 to a few KiB (small) or up to 200 KiB."""
    rng = streams.SplitMix(seed)
    out = bytearray()
    while len(out) < nbytes:
        r = rng.below(100)
        if r < 5:
            b0, plen = 0x89, rng.below(126)                 # ping
        else:
            b0 = (0x82, 0x81, 0x02, 0x80)[rng.below(4)]
            plen = rng.below(3000) if small else rng.below(200000)
        out += streams.header(b0, plen) + rng.bytes(plen)
    return bytes(out)


def check_vs_oracle(ws, oracle, src, **mode):
    view, _ = dev_bytes(src)
    ob = np.frombuffer(src, np.uint8).copy()
    ofr, carry, on = oracle.decode_stream(ob)
    dec = ws.frame_decoder(**mode)
    r = dec.decode(view, cap=on + 2)
    assert r.nframes == on
    assert host(view) == ob.tobytes()
    assert frames_list(r.frames(), True) == frames_list(ofr, True)
    assert carry_list(dec.carry()) == carry_list(carry)
    assert dec.ctx.last_device_error() == 0


@pytest.mark.parametrize("small_segments", [False, True])
@pytest.mark.parametrize("seed,nbytes,small", [(1, 3 << 20, True), (2, 24 << 20, False), (3, 5000, True)])
def test_unmasked_hint_server_streams(ws, oracle, seed, nbytes, small, small_segments):
    src = server_stream(seed, nbytes, small)
    check_vs_oracle(ws, oracle, src, small_segments=small_segments, opts=OPT_UNMASKED_HINT)
    # the same stream without the hint (client speculation, every entry implausible)
    check_vs_oracle(ws, oracle, src, small_segments=small_segments)


@pytest.mark.parametrize("name", ["random_frames_200", "tiny_frames", "fragments", "lengths", "random_bytes_3000"])
def test_wrong_hint_client_streams(ws, oracle, name):
    src = streams.case_bytes(name)
    for small_segments in (False, True):
        check_vs_oracle(ws, oracle, src, small_segments=small_segments, opts=OPT_UNMASKED_HINT)


def test_descriptor_region_overflow_and_truncation(ws, oracle):
    """Descriptor emission from the per-run frame-start regions: a run holding
    far more frames than the batch average overflows its region (the call
    falls back to re-walking the chains), and a caller capacity below the frame
    count truncates the table; both must equal the oracle's descriptors."""
    rng = streams.SplitMix(0xE417)
    out = bytearray()
    while len(out) < (48 << 20):  # large frames: few frames per run on average
        plen = 60000 + rng.below(8000)
        out += streams.header(0x82, plen, rng.bytes(4)) + rng.bytes(plen)
    for _ in range(40000):        # one dense stretch (~320 KiB): thousands of frames in one run
        plen = rng.below(2)
        out += streams.header(0x82, plen, rng.bytes(4)) + rng.bytes(plen)
    while len(out) < (64 << 20):
        plen = 60000 + rng.below(8000)
        out += streams.header(0x81, plen, rng.bytes(4)) + rng.bytes(plen)
    src = bytes(out)
    ob = np.frombuffer(src, np.uint8).copy()
    ofr, carry, on = oracle.decode_stream(ob)
    for cap in (on, on // 3):
        view, _ = dev_bytes(src)
        dec = ws.frame_decoder()
        r = dec.decode(view, cap=cap)
        assert r.nframes == on
        assert host(view) == ob.tobytes()
        assert frames_list(r.frames()[:cap], True) == frames_list(ofr[:cap], True)
        assert dec.ctx.last_device_error() == 0
