"""Deterministic WebSocket byte streams for parity tests.

Shared by gen_golden.py (which decodes them with the REAL reference, in the
survey container) and by the tests (which rebuild the same bytes on any box and
compare the GPU path / the oracle against the recorded reference output).
Randomness is splitmix64 in pure Python so the bytes never depend on a
library's RNG version.
"""
MASK64 = (1 << 64) - 1


class SplitMix:
    def __init__(self, seed):
        self.s = seed & MASK64

    def next(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & MASK64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        return z ^ (z >> 31)

    def below(self, n):
        return self.next() % n

    def bytes(self, n):
        out = bytearray()
        while len(out) < n:
            out += self.next().to_bytes(8, "little")
        return bytes(out[:n])


def header(b0, length, key=None, form=None, mask_bit=None):
    """Wire header. form: None = minimal (RFC), 7 / 16 / 64 = force a length form."""
    if form is None:
        form = 7 if length < 126 else (16 if length <= 0xFFFF else 64)
    mb = (key is not None) if mask_bit is None else mask_bit
    b1 = 0x80 if mb else 0
    if form == 7:
        out = bytes([b0, b1 | (length & 0x7F)])
    elif form == 16:
        out = bytes([b0, b1 | 126]) + (length & 0xFFFF).to_bytes(2, "big")
    else:
        out = bytes([b0, b1 | 127]) + (length & MASK64).to_bytes(8, "big")
    if key is not None:
        out += bytes(key)
    return out


def masked(payload, key):
    return bytes(b ^ key[i % 4] for i, b in enumerate(payload))


def frame(rng, b0, plen, masked_frame=True, form=None):
    key = rng.bytes(4) if masked_frame else None
    pl = rng.bytes(plen)
    return header(b0, plen, key, form) + (masked(pl, key) if masked_frame else pl)


def case_bytes(name):
    """Named edge-case streams."""
    rng = SplitMix(sum(name.encode()) * 1000003 + len(name))
    if name == "rfc_hello":
        return bytes.fromhex("818537fa213d7f9f4d5158")
    if name == "empty":
        return b""
    if name == "lengths":
        return b"".join(frame(rng, 0x82, n) for n in
                        (0, 1, 2, 3, 4, 5, 125, 126, 127, 300, 65535, 65536, 65537, 7, 0))
    if name == "unmasked_mix":
        return b"".join(frame(rng, b0, n, masked_frame=(i % 2 == 0)) for i, (b0, n) in
                        enumerate([(0x81, 10), (0x82, 200), (0x01, 3), (0x80, 0), (0x82, 70000),
                                   (0x89, 4), (0x8A, 0), (0x82, 33)]))
    if name == "rsv_reserved_ops":
        return b"".join(frame(rng, b0, n) for b0, n in
                        [(0xF1, 9), (0xC3, 17), (0x94, 1), (0x87, 130), (0x8B, 2), (0x0F, 5),
                         (0x82, 12)])
    if name == "bad_control":
        return b"".join(frame(rng, b0, n) for b0, n in
                        [(0x08, 2), (0x88, 126), (0x89, 200), (0x0A, 0), (0x82, 8)])
    if name == "nonminimal":
        return (frame(rng, 0x82, 5, form=16) + frame(rng, 0x82, 200, form=64) +
                frame(rng, 0x82, 0, form=16) + frame(rng, 0x81, 125, form=64) +
                frame(rng, 0x82, 65535, form=64) + frame(rng, 0x82, 9))
    if name == "len_msb":  # 64-bit length with MSB set: swallows the rest of the batch
        return frame(rng, 0x82, 40) + header(0x82, (1 << 63) + 1, rng.bytes(4)) + rng.bytes(500)
    if name == "huge_len_eats_tail":
        return frame(rng, 0x82, 3) + header(0x82, 1 << 40, rng.bytes(4)) + rng.bytes(777)
    if name.startswith("trunc_hdr_"):  # a 14-byte header cut after k bytes
        k = int(name.rsplit("_", 1)[1])
        return frame(rng, 0x82, 100) + header(0x82, 70000, rng.bytes(4))[:k]
    if name == "trunc_payload":
        return frame(rng, 0x82, 50) + frame(rng, 0x82, 5000)[:2000]
    if name == "fragments":
        out = b""
        for i in range(6):
            b0 = (0x01 if i == 0 else 0x00) | (0x80 if i == 5 else 0)
            out += frame(rng, b0, rng.below(3000))
            if i == 2:
                out += frame(rng, 0x89, 10)
        return out
    if name == "tiny_frames":
        return b"".join(frame(rng, 0x82, rng.below(6)) for _ in range(700))
    if name == "small_frames_4k":
        return b"".join(frame(rng, 0x82, 256) for _ in range(300))
    if name.startswith("random_bytes_"):  # arbitrary bytes are a valid input too
        n = int(name.rsplit("_", 1)[1])
        return rng.bytes(n)
    if name.startswith("random_frames_"):  # random plausible-ish headers, mixed forms
        n = int(name.rsplit("_", 1)[1])
        out = b""
        for _ in range(n):
            r = rng.below(100)
            b0 = rng.below(256) if r < 10 else (0x80 | [0, 1, 2, 8, 9, 10][rng.below(6)])
            plen = [rng.below(126), 126 + rng.below(1000), 65536 + rng.below(70000),
                    rng.below(8)][rng.below(4)]
            form = None if r >= 5 else [7, 16, 64][rng.below(3)]
            if form == 7:
                plen &= 0x7F
                plen = min(plen, 125)
            out += frame(rng, b0, plen, masked_frame=(r < 95), form=form)
        return out
    raise KeyError(name)


EDGE_CASES = (["rfc_hello", "empty", "lengths", "unmasked_mix", "rsv_reserved_ops",
               "bad_control", "nonminimal", "len_msb", "huge_len_eats_tail", "trunc_payload",
               "fragments", "tiny_frames", "small_frames_4k"] +
              [f"trunc_hdr_{k}" for k in range(1, 14)] +
              ["random_bytes_64", "random_bytes_3000", "random_bytes_100000",
               "random_frames_40", "random_frames_200"])
