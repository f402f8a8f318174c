#!/usr/bin/env python3
"""Expected outputs of the §8(f) callers on the full benchmark batches, for
`bench.py --op encode|classify|reassemble` (tests/golden/ops.json).

CONTAINER-ONLY test infrastructure: runs the committed restatement
(oracle/xyws_oracle.c: oracle_encode_frames, oracle_classify,
oracle_reassemble), whose builder is pinned by the reference's own header
bytes (frame_header.json, tests/test_oracle.py) and whose stream decode is
pinned by configs.json (the reference's digests), on the same synthetic
batches (include/xyws_synth.h). The reference has no batched encode,
classification or reassembly to run: these digests are the restatement's
(parity for these ops is pinned only through its builder and decode).

Re-run with:  python tests/golden/gen_ops_golden.py
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from oracle.oracle import Oracle, Carry, _ptr  # noqa: E402

# the bench's op parameters (bench.py OP_PARAMS must match)
ENC_FLAGS = 0x11         # echo_once: FIN | TEXT, unmasked (websocket_echo.cpp:22)
CLS_MAX_PAYLOAD = 1 << 20
CLS_POLICY = 0x1         # XYWS_POL_FRAGMENTS
RS_OPTS = 0x1            # XYWS_REASM_UTF8

CONFIGS = {
    "c1_text_4k": ("uniform", 65536, 4096, 0x81, 0x5EED0001),
    "c2_bin_256": ("uniform", 1 << 20, 256, 0x82, 0x5EED0002),
    "c3_bin_64k": ("uniform", 32768, 65536, 0x82, 0x5EED0003),
    "c4_mixed": ("mixed", None, 1 << 30, None, 0x5EED0004),
}


def main():
    orc = Oracle()
    L = orc.L
    out = {}
    only = sys.argv[1:]
    for name, (kind, n, p, b0, seed) in CONFIGS.items():
        if only and name not in only:
            continue
        t0 = time.time()
        if kind == "uniform":
            buf = orc.fill_uniform(n, p, b0, seed)
        else:
            tab, nf, total = orc.mixed_table(seed, p)
            buf = orc.fill_mixed(tab, nf, total, seed)
            n = nf
        raw, cout, nd = orc.decode_stream_raw(buf, n + 2)  # buf now holds the decoded batch
        fr = raw.ctypes.data
        rec = {"frames": int(nd)}
        # encode: echo replies for every frame
        total = L.oracle_encode_frames(_ptr(buf), buf.size, fr, nd, ENC_FLAGS, 0, None, None, 0, None, 0, None)
        enc = np.zeros(max(total, 1), np.uint8)
        L.oracle_encode_frames(_ptr(buf), buf.size, fr, nd, ENC_FLAGS, 0, None, None, 0, _ptr(enc), total, None)
        rec["encode"] = {"flags": ENC_FLAGS, "out_len": int(total), "out_digest": orc.digest(enc[:total])}
        del enc
        # classify
        verd = np.zeros(max(nd, 1) * 8, np.uint8)
        first = C.c_uint64()
        L.oracle_classify(_ptr(buf), buf.size, fr, nd, CLS_MAX_PAYLOAD, CLS_POLICY, _ptr(verd), C.byref(first))
        rec["classify"] = {"max_payload": CLS_MAX_PAYLOAD, "policy": CLS_POLICY,
                           "verdicts_digest": orc.digest(verd[:nd * 8]), "first_close": first.value}
        # reassemble (+ UTF-8)
        plen = np.frombuffer(raw.tobytes(), dtype=np.uint64).reshape(-1, 4)[:, 2]
        cap = int(plen.sum())
        rs = np.zeros(max(cap, 1), np.uint8)
        msgs = np.zeros(max(nd, 1) * 40, np.uint8)
        nm = L.oracle_reassemble(_ptr(buf), buf.size, fr, nd, RS_OPTS, _ptr(rs), cap, _ptr(msgs), nd)
        rec["reassemble"] = {"opts": RS_OPTS, "out_cap": cap, "messages": int(nm),
                             "out_digest": orc.digest(rs[:cap]), "msgs_digest": orc.digest(msgs[:nm * 40])}
        out[name] = rec
        del buf, rs, msgs
        print(f"  {name}: {nd} frames, {time.time() - t0:.1f}s", flush=True)
    path = os.path.join(HERE, "ops.json")
    if only and os.path.exists(path):
        old = json.load(open(path))["configs"]
        old.update(out)
        out = old
    with open(path, "w") as f:
        json.dump({"configs": out}, f, indent=1, sort_keys=True)
    print("wrote ops.json")


if __name__ == "__main__":
    main()
