"""The loopback echo harness (examples/echo_loopback.cpp): the reference's
echo server (example/websocket/websocket_echo.cpp:18-27 with the close policy
of example/include/common/websocket.h:81-108) over a real 127.0.0.1 TCP
connection, decoding / classifying / encoding each recv batch on the GPU.
The harness checks the whole reply stream byte for byte against the replies
the reference's echo sends (FIN|TEXT echo per frame, a close frame with the
first close code) and exits non-zero on any difference.
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
def test_echo_pings_get_pongs():
    j = run("--frames", 4000, "--ping-every", 7, "--chunk", 4096)
    assert j["ok"] and j["close_code"] == 1000


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [512, 65536])
def test_echo_oversize_frame_closes_1009(chunk):
    j = run("--frames", 2000, "--oversize", "--chunk", chunk)
    assert j["ok"] and j["close_code"] == 1009 and j["frames"] == 1999


@pytest.mark.gpu
def test_echo_small_receive_buffer():
    # a 4 KiB receive buffer: frames straddle nearly every batch
    j = run("--frames", 3000, "--buf", 4096, "--chunk", 65536)
    assert j["ok"] and j["close_code"] == 1000
