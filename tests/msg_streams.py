"""Client streams with messages for the tests of the callers either side of the
decode path (xyws_encode_frames / xyws_classify_frames / xyws_reassemble):
fragmented text and binary messages, control frames between fragments, close
frames with status codes, orphan continuations, interrupted messages and
invalid UTF-8. Deterministic (splitmix64 via tests/golden/streams.py)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import streams  # noqa: E402

TEXTS = ["hello", "héllo wörld", "€ 𝄞 ✓ 日本語", "", "a" * 300, "Grüße, ünïcödé " * 40]
BAD_UTF8 = [b"\xc0\xaf", b"\xed\xa0\x80", b"\xe0\x80\x80", b"\xf4\x90\x80\x80", b"\xff", b"abc\x80",
            b"\xe2\x82\xac\x82", b"\xf0\x9f\x98"]


def _frame(rng, b0, payload, masked=True):
    key = rng.bytes(4) if masked else None
    return streams.header(b0, len(payload), key) + (streams.masked(payload, key) if masked else payload)


def split_parts(rng, data, k):
    """data cut into k parts at random points (parts may be empty)."""
    cuts = sorted(rng.below(len(data) + 1) for _ in range(k - 1))
    out, prev = [], 0
    for c in cuts + [len(data)]:
        out.append(data[prev:c])
        prev = c
    return out


def message_stream(seed, nmsg=40, bad=True, orphans=True, interrupted=True, unmasked=False):
    """Bytes of a client stream: (wire bytes, list of (opcode, payload) of every
    COMPLETE message in order)."""
    rng = streams.SplitMix(seed)
    out, msgs = b"", []
    for m in range(nmsg):
        r = rng.below(100)
        text = r < 60
        if text:
            if bad and rng.below(6) == 0:
                pl = TEXTS[rng.below(len(TEXTS))].encode() + BAD_UTF8[rng.below(len(BAD_UTF8))]
            else:
                pl = TEXTS[rng.below(len(TEXTS))].encode()
        else:
            pl = rng.bytes(rng.below(2000))
        op = 1 if text else 2
        k = 1 + rng.below(4)
        parts = split_parts(rng, pl, k)
        cut = False
        for i, p in enumerate(parts):
            b0 = (op if i == 0 else 0) | (0x80 if i == k - 1 else 0)
            cut = interrupted and k > 1 and i == k - 1 and rng.below(12) == 0
            if cut:
                break  # the FIN fragment never comes: a new message interrupts this one
            out += _frame(rng, b0, p, masked=not (unmasked and rng.below(5) == 0))
            if i < k - 1 and rng.below(4) == 0:
                out += _frame(rng, 0x89, rng.bytes(rng.below(20)))  # a ping between fragments
        else:
            msgs.append((op, pl))
        if orphans and not cut and rng.below(15) == 0:
            out += _frame(rng, 0x80, rng.bytes(rng.below(50)))  # a continuation outside a message
        if rng.below(10) == 0:
            out += _frame(rng, 0x8A, rng.bytes(rng.below(10)))  # an unsolicited pong
    return out, msgs


def close_frame(rng, code=None, reason=b""):
    pl = b"" if code is None else code.to_bytes(2, "big") + reason
    return _frame(rng, 0x88, pl)
