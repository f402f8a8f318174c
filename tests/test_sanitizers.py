"""Host-side sanitizer run: the C restatement built with
AddressSanitizer + UndefinedBehaviorSanitizer (oracle/Makefile,
liboracle_asan.so) driven over the reference's golden corpus in a child
process with libasan preloaded: the parser (whole, byte-at-a-time), the mask
at every phase, stream decodes of every edge case split at every golden
point with the carry, and the multithreaded batch decode. Any ASan report or
UBSan error aborts the child (-fno-sanitize-recover), failing the test. CPU
only; sanitizers never run on GPU code here.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")

CHILD = r"""
import json, os, sys
import numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, os.path.join(sys.argv[1], "tests", "golden"))
from oracle.oracle import Oracle
import streams
orc = Oracle(os.path.join(sys.argv[1], "oracle", "liboracle_asan.so"))
G = lambda n: json.load(open(os.path.join(sys.argv[1], "tests", "golden", n)))
for c in G("parse_corpus.json")["corpus"]:
    hb = bytes.fromhex(c["bytes"])
    p = orc.parser()
    assert p.parse(hb) == c["ret"]
    q = orc.parser()
    assert [q.parse(hb[i:i + 1]) for i in range(len(hb))] == c["feed"]
for ph in range(4):
    a = np.frombuffer(bytes(range(256)) * 3, np.uint8).copy()
    orc.mask(a[ph:], 0x04030201, ph)
cases = G("streams.json")["cases"]
for name in streams.EDGE_CASES:
    src = streams.case_bytes(name)
    b = np.frombuffer(src, np.uint8).copy() if src else np.zeros(0, np.uint8)
    fr, carry, n = orc.decode_stream(b)
    assert n == cases[name]["nframes"], name
    for s in cases[name].get("splits", []):
        k = s["k"]
        x = np.frombuffer(src[:k], np.uint8).copy() if k else np.zeros(0, np.uint8)
        y = np.frombuffer(src[k:], np.uint8).copy() if k < len(src) else np.zeros(0, np.uint8)
        _, c1, n1 = orc.decode_stream(x)
        _, c2, n2 = orc.decode_stream(y, carry_in=c1)
        assert n1 + n2 == cases[name]["nframes"], (name, k)
big = np.frombuffer(streams.case_bytes("random_frames_200"), np.uint8).copy()
orc.decode_batch_mt(big, 4)
print("sanitized ok")
"""


def _libasan():
    r = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True)
    path = r.stdout.strip()
    return path if r.returncode == 0 and os.path.isabs(path) and os.path.exists(path) else None


def test_restatement_under_asan_ubsan():
    asan = _libasan()
    if asan is None:
        pytest.skip("libasan not available")
    r = subprocess.run(["make", "-C", ORACLE, "liboracle_asan.so"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    env = dict(os.environ)
    env["LD_PRELOAD"] = asan
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0 and "sanitized ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
