"""The C++ boundary: include/xyws/websocket.hpp (xynet's class names over the
C-ABI) used from C++.

- CPU: the shim compiles standalone with g++ -std=c++20 for a websocket.h-
  shaped caller (parse -> result -> websocket_mask), and xyws_header_build
  (the reference builder, websocket_frame_header.h:136-175) reproduces the
  reference's own header bytes (frame_header.json builds, from oracle/_ref).
- GPU: tests/cpp/test_shim (built by __graft_entry__.build()) runs the header
  round trip of test/websocket_frame_test.cpp:10-65 (9 cases), the every-byte
  split parse of :67-89, the builder vectors and a device receive loop, all
  through the shim, with the expected values of frame_header.json.
"""
import ctypes as C
import os
import subprocess

import pytest

from conftest import load_golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "test_shim")

CALLER = r'''
#include "xyws/websocket.hpp"
// websocket_recv_data's loop (example/include/common/websocket.h:110-134)
// against the shim alone
std::span<std::byte> recv_data(xyws::context& ctx, std::span<std::byte> dev_buf, std::size_t recv_bytes) {
  auto parser = xyws::websocket_frame_header_parser{ctx};
  auto ret = parser.parse(std::span{dev_buf.data(), recv_bytes});
  if (ret == xyws::websocket_frame_header_parser::npos) return {};
  auto [flags, mask, length] = parser.result();
  (void)flags;
  auto data_span = std::span{dev_buf.data() + ret, length};
  xyws::websocket_mask(ctx, data_span, mask, 0);
  return data_span;
}
int main() {
  auto header = xyws::websocket_frame_header{xyws::websocket_flags::WS_FINAL_FRAME | xyws::websocket_flags::WS_OP_TEXT, 5};
  return (int)header.span().size() - 2;
}
'''


def vectors_text():
    g = load_golden("frame_header.json")
    lines = []
    for c in g["cases"]:
        lines.append(f"case {c['flags']} {c['length']} {c['header']} {c['ret']} {c['r_flags']} {c['r_length']}")
    for s in g["splits"]:  # test2: FIN | HAS_MASK | PING, length 120 (websocket_frame_test.cpp:69-73)
        lines.append(f"split 57 120 {s['split']} {s['ret1']} {s['ret2']} {s['r_flags']} {s['r_length']}")
    for b in g["builds"]:
        lines.append(f"build {b['flags']} {b['length']} {b['key']} {b['built_nokey']} {b['ctor_masked']} {b['built']}")
    return "\n".join(lines) + "\n"


def test_shim_compiles_for_a_websocket_h_caller(tmp_path):
    src = tmp_path / "caller.cpp"
    src.write_text(CALLER)
    r = subprocess.run(["g++", "-std=c++20", "-Wall", "-Werror", "-fsyntax-only", "-I", os.path.join(ROOT, "include"),
                        str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_header_build_matches_reference_builds():
    from xynet_amd import _lib
    L = _lib.load()
    g = load_golden("frame_header.json")
    for b in g["builds"]:
        out = (C.c_uint8 * 16)()
        n = L.xyws_header_build(b["flags"], None, b["length"], out)
        assert bytes(out[:n]).hex() == b["built_nokey"] == b["ctor_masked"]
        key = (C.c_uint8 * 4)(*bytes.fromhex(b["key"]))
        n = L.xyws_header_build(b["flags"], key, b["length"], out)
        assert bytes(out[:n]).hex() == b["built"]
        assert n == b["size"]


def test_python_header_class_keeps_the_masked_ctor_quirk():
    from xynet_amd import websocket as ws
    g = load_golden("frame_header.json")
    for b in g["builds"]:
        h = ws.websocket_frame_header(b["flags"], b["length"], mask=bytes.fromhex(b["key"]))
        assert h.span().hex() == b["ctor_masked"]


@pytest.mark.gpu
def test_cpp_shim_program_on_device(tmp_path):
    assert os.path.exists(BIN), "tests/cpp/test_shim not built (run __graft_entry__.build())"
    vec = tmp_path / "vectors.txt"
    vec.write_text(vectors_text())
    r = subprocess.run([BIN, str(vec)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    n = 9 + len(load_golden("frame_header.json")["splits"]) + len(load_golden("frame_header.json")["builds"])
    assert f"ok {n}" in r.stdout, r.stdout


COMPAT_SRC = os.path.join(ROOT, "tests", "cpp", "test_compat.cpp")
COMPAT_BIN = os.path.join(ROOT, "tests", "cpp", "test_compat")


def test_websocket_h_caller_switches_by_include():
    """websocket_recv_data in shape (websocket.h:110-134: `using namespace
    xynet`, websocket_frame_header_parser{}, the three-argument
    websocket_mask of websocket_frame_mask.h:14) compiles against the shim."""
    r = subprocess.run(["g++", "-std=c++20", "-Wall", "-Werror", "-fsyntax-only", "-I", os.path.join(ROOT, "include"),
                        COMPAT_SRC], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_websocket_h_caller_on_device():
    """The same program run: 32 frames (0-1000 B payloads, received in pieces
    of 14-1024 B) parsed and unmasked from host buffers, plus the
    three-argument mask at phase 6 (its return i + len)."""
    assert os.path.exists(COMPAT_BIN), "tests/cpp/test_compat not built (run __graft_entry__.build())"
    r = subprocess.run([COMPAT_BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok 35" in r.stdout, r.stdout
