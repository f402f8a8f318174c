"""The loopback echo harness (examples/echo_loopback.cpp): the reference's
echo server (example/websocket/websocket_echo.cpp:18-27 with the close policy
of example/include/common/websocket.h:81-108) over a real 127.0.0.1 TCP
connection, decoding / classifying / encoding each recv batch on the GPU.
The harness checks the whole reply stream byte for byte against the replies
the reference's echo sends (FIN|TEXT echo per frame, a close frame with the
first close code) and exits non-zero on any difference. By default the server
is the reference's, its bit-3 close test included (websocket.h:87: a ping
closes 1000); `--rfc` is an RFC 6455 server instead (pings answered with
pongs), a deliberate departure from the reference tested on its own.
"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "examples", "echo_loopback")


def test_echo_harness_is_built():
    assert os.access(BIN, os.X_OK), "run __graft_entry__.build() first"


def run(*args):
    r = subprocess.run([BIN, *map(str, args)], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [1, 37, 1000, 65536, 1 << 20])
def test_echo_replies_match_reference_echo(chunk):
    # chunk = the client's write size: 1-byte writes cut every header and
    # payload at every position across recv batches
    frames = 300 if chunk < 100 else 5000
    j = run("--frames", frames, "--chunk", chunk, "--seed", 0x5EED0001 + chunk)
    assert j["ok"] and j["close_code"] == 1000 and j["frames"] == frames


@pytest.mark.gpu
def test_echo_ping_closes_1000_like_the_reference():
    # websocket.h:87 tests `flags & WS_OP_CLOSE`, bit 3 of the opcode: the
    # reference's echo answers the first ping (0x9) with close 1000, and every
    # frame before it with a FIN|TEXT echo
    j = run("--frames", 4000, "--ping-every", 7, "--chunk", 4096)
    assert j["ok"] and j["close_code"] == 1000 and j["frames"] == 6 and j["mode"] == "reference"


@pytest.mark.gpu
def test_echo_rfc_mode_pings_get_pongs():
    # --rfc departs from the reference on purpose: pongs for pings
    j = run("--frames", 4000, "--ping-every", 7, "--chunk", 4096, "--rfc")
    assert j["ok"] and j["close_code"] == 1000 and j["mode"] == "rfc"


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [512, 65536])
def test_echo_oversize_frame_closes_1009(chunk):
    j = run("--frames", 2000, "--oversize", "--chunk", chunk)
    assert j["ok"] and j["close_code"] == 1009 and j["frames"] == 1999


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [4096, 65536])
def test_echo_oversize_header_closes_before_its_payload(chunk):
    # a header announcing 200 000 B (far past the 4 KiB receive buffer): the
    # reference closes 1009 on the header (websocket.h:102-105), before the
    # payload arrives; the server must not wait for it
    j = run("--frames", 500, "--oversize", "--oversize-len", 200000, "--buf", 4096, "--chunk", chunk)
    assert j["ok"] and j["close_code"] == 1009 and j["frames"] == 499 and j["closed_on_header"]


@pytest.mark.gpu
def test_echo_small_receive_buffer():
    # a 4 KiB receive buffer: frames straddle nearly every batch
    j = run("--frames", 3000, "--buf", 4096, "--chunk", 65536)
    assert j["ok"] and j["close_code"] == 1000
