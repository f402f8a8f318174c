#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/ from the REAL reference.

CONTAINER-ONLY: needs oracle/_ref/libxynet_ref.so, which oracle/Makefile builds
from the reference headers in /root/reference/include (see
oracle/ref_harness.cpp). The GPU box never runs this; it only reads the JSON
files it wrote. Re-run with:  python tests/golden/gen_golden.py

Files written (all data: inputs are rebuilt by tests/golden/streams.py or by
the synthetic-batch spec include/xyws_synth.h; expected outputs are the
reference's):
  frame_header.json  reference test cases (test/websocket_frame_test.cpp:10-89)
                     + builder/size tables (websocket_frame_header.h:111-224)
  parse_corpus.json  header byte strings -> parse()/result(), whole and
                     byte-at-a-time (websocket_frame_header.h:305-385)
  unmask.json        websocket_mask vectors (websocket_frame_mask.h:6-25)
  streams.json       edge-case streams -> decoded bytes, frames, carries, and
                     carries at split points
  configs.json       digests of the full benchmark batches before/after the
                     reference decode
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from oracle.oracle import Oracle, Reference, Carry, Frame, NPOS  # noqa: E402
import streams  # noqa: E402

FIN, MASK, PING = 0x10, 0x20, 0x09


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
    print("wrote", name, os.path.getsize(os.path.join(HERE, name)), "bytes")


def gen_frame_header(ref):
    # test/websocket_frame_test.cpp:15-57 subcases (flags, length)
    sub = [(0, 0), (0, 120), (0, 126), (0, 0xFFFF - 1234), (0, 0xFFFF + 1), (FIN, 120),
           (MASK, 0xFFFFFFFF), (FIN | MASK | PING, 120), (0, 0xFFFFFFFF)]
    cases = []
    for flags, length in sub:
        hb = ref.header_ctor(flags, length)
        p = ref.parser()
        ret = p.parse(hb)
        f, m, l = p.result()
        cases.append(dict(flags=flags, length=length, header=hb.hex(), ret=ret, r_flags=f,
                          r_mask=m, r_length=l))
    # test2 (:67-89): split the FIN|MASK|PING, 120 header at every byte
    hb = ref.header_ctor(FIN | MASK | PING, 120)
    splits = []
    for k in range(len(hb)):
        p = ref.parser()
        r1 = p.parse(hb[:k])
        r2 = p.parse(hb[k:])
        f, m, l = p.result()
        splits.append(dict(split=k, ret1=r1, ret2=r2, r_flags=f, r_length=l))
    # builder with key bytes and the masked ctor quirk (key bytes stay zero, a4)
    rng = streams.SplitMix(7)
    builds = []
    for flags in (0, FIN, MASK, FIN | MASK | 1, FIN | MASK | 2, MASK | 8, 0x0F | FIN | MASK):
        for length in (0, 1, 125, 126, 127, 0xFFFF, 0x10000, 0xFFFFFFFF, 1 << 40, (1 << 64) - 1):
            key = rng.bytes(4)
            builds.append(dict(flags=flags, length=length, key=key.hex(),
                               built=ref.header_build(flags, key, length).hex(),
                               built_nokey=ref.header_build(flags, None, length).hex(),
                               ctor_masked=ref.header_ctor(flags, length,
                                                           int.from_bytes(key, "little")).hex(),
                               size=ref.calc_frame_header_size(flags, length)))
    dump("frame_header.json", dict(cases=cases, splits=splits, builds=builds,
                                   max_header_size=ref.calc_frame_header_size(MASK, 0xFFFFFFFF)))


def gen_parse_corpus(ref):
    rng = streams.SplitMix(11)
    corpus = [bytes.fromhex(h) for h in (
        "8105", "818537fa213d7f9f4d5158", "82fe0005aabbccdd", "82ff8000000000000001aabbccdd",
        "f180aabbccdd", "8380aabbccdd", "008aaabbccdd", "88", "", "80", "827e", "827f00",
        "827f0000000000010000", "02fe0100", "89ff00000000000000ffdeadbeef")]
    for _ in range(120):
        b0 = rng.below(256)
        l7 = [rng.below(126), 126, 127][rng.below(3)]
        b1 = l7 | (0x80 if rng.below(4) else 0)
        ext = rng.bytes(2 if l7 == 126 else 8 if l7 == 127 else 0)
        key = rng.bytes(4) if b1 & 0x80 else b""
        tail = rng.bytes(rng.below(5))
        corpus.append(bytes([b0, b1]) + ext + key + tail)
    out = []
    for hb in corpus:
        p = ref.parser()
        ret = p.parse(hb)
        f, m, l = p.result()
        again = p.parse(hb) if len(hb) else NPOS  # after s_finished: npos until reset
        q = ref.parser()
        feed = [q.parse(hb[i:i + 1]) for i in range(len(hb))]
        fq, mq, lq = q.result()
        out.append(dict(bytes=hb.hex(), ret=ret, flags=f, mask=m, length=l, again=again,
                        feed=feed, feed_flags=fq, feed_mask=mq, feed_length=lq))
    dump("parse_corpus.json", dict(corpus=out))


def gen_unmask(ref):
    lens = list(range(0, 68)) + [255, 256, 257, 4095, 4096, 4097, 65535, 65536, 65537, 1 << 20]
    vecs = []
    for n in lens:
        for phase in (0, 1, 2, 3, 5, 1 << 33):
            rng = streams.SplitMix(n * 131 + phase)
            key = rng.next() & 0xFFFFFFFF
            data = np.frombuffer(rng.bytes(n), np.uint8).copy() if n else np.zeros(0, np.uint8)
            seed = n * 131 + phase
            ret = ref.mask(data, key, phase)
            rec = dict(n=n, phase=phase, key=key, seed=seed, ret=ret)
            if n <= 300:
                rec["out"] = data.tobytes().hex()
            else:
                rec["out_digest"] = Oracle().digest(data)
            vecs.append(rec)
    dump("unmask.json", dict(vectors=vecs))


def frames_json(frames):
    return [[f.frame_off, f.payload_off, f.payload_len, bytes(f.key).hex(), f.flags, f.hdr_len,
             f.status & 0x01] for f in frames]


def carry_json(c):
    return [c.payload_remaining, c.phase, c.frames_total, bytes(c.key).hex(), c.hdr_len,
            bytes(c.hdr[:c.hdr_len]).hex()]


def gen_streams(ref, orc):
    cases = {}
    for name in streams.EDGE_CASES:
        src = streams.case_bytes(name)
        buf = np.frombuffer(src, np.uint8).copy() if src else np.zeros(0, np.uint8)
        frames, cout, n = ref.decode_stream(buf)
        rec = dict(size=len(src), in_digest=orc.digest(np.frombuffer(src, np.uint8)) if src
                   else orc.digest(np.zeros(0, np.uint8)),
                   nframes=n, frames=frames_json(frames), carry=carry_json(cout))
        if len(src) <= 8192:
            rec["out"] = buf.tobytes().hex()
        rec["out_digest"] = orc.digest(buf)
        # split points: decode [0,k) then [k,len) with the carry; record mid carry
        L = len(src)
        if L <= 300:
            pts = list(range(0, L + 1))
        else:
            rng = streams.SplitMix(L)
            pts = sorted(set([0, 1, L - 1, L] + [rng.below(L + 1) for _ in range(40)] +
                             [f.frame_off + d for f in frames[:20] for d in (0, 1, 2, 5, 9, 13)
                              if 0 <= f.frame_off + d <= L]))
        splits = []
        for k in pts:
            a = np.frombuffer(src[:k], np.uint8).copy() if k else np.zeros(0, np.uint8)
            b = np.frombuffer(src[k:], np.uint8).copy() if k < L else np.zeros(0, np.uint8)
            fa, ca, na = ref.decode_stream(a)
            fb, cb, nb = ref.decode_stream(b, carry_in=ca)
            joined = np.concatenate([a, b])
            assert orc.digest(joined) == rec["out_digest"], (name, k)
            assert na + nb == n and carry_json(cb)[:3] == carry_json(cout)[:3], (name, k)
            splits.append(dict(k=k, n1=na, carry_mid=carry_json(ca)))
        rec["splits"] = splits
        cases[name] = rec
    dump("streams.json", dict(cases=cases))


CONFIGS = {
    # name: (kind, nframes, payload, b0, seed) — SURVEY.md §8(d)
    "c1_text_4k": ("uniform", 65536, 4096, 0x81, 0x5EED0001),
    "c2_bin_256": ("uniform", 1 << 20, 256, 0x82, 0x5EED0002),
    "c3_bin_64k": ("uniform", 32768, 65536, 0x82, 0x5EED0003),
    "c4_mixed": ("mixed", None, 1 << 30, None, 0x5EED0004),
}
for g in range(8):
    CONFIGS[f"c5_shard{g}"] = ("uniform", 32768, 65536, 0x82, 0x5EED0005 + g)
# small uniform batches the CPU-side tests can afford
CONFIGS["t_bin_64k_x64"] = ("uniform", 64, 65536, 0x82, 0x5EED0003)
CONFIGS["t_bin_256_x4096"] = ("uniform", 4096, 256, 0x82, 0x5EED0002)
CONFIGS["t_mixed_8m"] = ("mixed", None, 8 << 20, None, 0x5EED0004)


def gen_configs(ref, orc, only=None):
    out = {}
    for name, (kind, n, p, b0, seed) in CONFIGS.items():
        if only and name not in only:
            continue
        t0 = time.time()
        if kind == "uniform":
            buf = orc.fill_uniform(n, p, b0, seed)
            rec = dict(kind=kind, nframes=n, payload=p, b0=b0, seed=seed)
        else:
            tab, nf, total = orc.mixed_table(seed, p)
            buf = orc.fill_mixed(tab, nf, total, seed)
            rec = dict(kind=kind, target=p, seed=seed, nframes=nf)
        rec["size"] = int(buf.size)
        rec["in_digest"] = orc.digest(buf)
        nmax = n if n is not None else nf
        raw, cout, nd = ref.decode_stream_raw(buf, nmax)
        assert nd == nmax, (name, nd, nmax)
        rec["decoded_frames"] = nd
        rec["out_digest"] = orc.digest(buf)
        rec["carry"] = carry_json(cout)
        first = (Frame * 4).from_buffer_copy(raw[:4 * 32].tobytes())
        rec["first_frames"] = frames_json(list(first))
        # the whole descriptor table the reference produced (what a
        # websocket_recv_data caller consumes, websocket.h:110-134)
        rec["frames_digest"] = orc.frames_digest(raw)
        out[name] = rec
        del buf
        print(f"  {name}: {rec['size']} B, {nd} frames, {time.time() - t0:.1f}s")
    dump("configs.json", dict(configs=out))


def main():
    ref = Reference("O2")
    orc = Oracle()
    if "--configs" in sys.argv:  # only configs.json
        gen_configs(ref, orc)
        return
    gen_frame_header(ref)
    gen_parse_corpus(ref)
    gen_unmask(ref)
    gen_streams(ref, orc)
    gen_configs(ref, orc)


if __name__ == "__main__":
    main()
