"""CPU checks of the drop-in boundary: the C-ABI library loads, exports every
function include/xyws.h declares, keeps the struct layouts, and fails loudly
(no CPU fallback) when no device is present."""
import ctypes as C
import os
import subprocess

import pytest

import xynet_amd._lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    lib = L.load()
    names = L.declared_symbols()
    assert "xyws_decode_stream" in names and "xyws_unmask" in names
    for n in names:
        assert hasattr(lib, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", L.lib_path()], capture_output=True,
                         text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(names) <= exported


def test_tools_library_exports():
    t = L.load_tools()
    for n in ("xyws_tools_fill_uniform", "xyws_tools_fill_mixed", "xyws_tools_digest",
              "xyws_tools_mixed_table"):
        assert hasattr(t, n)


def test_library_is_gfx950_code_object():
    data = open(L.lib_path(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data or b"gfx950" in data


def test_struct_layouts_match_header():
    assert C.sizeof(L.Frame) == 32 and C.sizeof(L.Carry) == 64
    off = {f[0]: getattr(L.Frame, f[0]).offset for f in L.Frame._fields_}
    assert off["payload_len"] == 16 and off["key"] == 24 and off["status"] == 30
    coff = {f[0]: getattr(L.Carry, f[0]).offset for f in L.Carry._fields_}
    assert coff["key"] == 24 and coff["hdr_len"] == 28 and coff["hdr"] == 29


def test_abi_version_and_strerror():
    lib = L.load()
    assert lib.xyws_abi_version() == 2
    assert lib.xyws_strerror(0) == b"ok"
    assert lib.xyws_strerror(-2) == b"HIP runtime error"


def test_null_arguments_rejected():
    lib = L.load()
    assert lib.xyws_ctx_create(0, None) == -1
    assert lib.xyws_unmask(None, None, 0, None, 0, None, None) == -1
    assert lib.xyws_decode_stream(None, None, 0, None, None, None, 0, None, 0, None) == -1
    assert lib.xyws_decode_indexed(None, None, 0, None, 0, None, 0, None) == -1


def test_no_device_fails_loudly():
    """Without a GPU the context cannot be created: no silent host fallback."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    lib = L.load()
    h = C.c_void_p()
    assert lib.xyws_ctx_create(0, C.byref(h)) == -2
    from xynet_amd import websocket as ws
    with pytest.raises(L.XywsError):
        ws.Context(0)


def test_product_does_not_reference_oracle():
    """The shipped path never links or imports the oracle."""
    for root, _, files in os.walk(os.path.join(ROOT, "xynet_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                src = open(os.path.join(root, f)).read()
                assert "oracle" not in src.replace("oracle/", "").lower() or f == "build.py", f
    out = subprocess.run(["ldd", L.lib_path()], capture_output=True, text=True).stdout
    assert "oracle" not in out and "xynet_ref" not in out


SHIM_PROG = r"""
#include <cstdio>
#include "xyws/websocket.hpp"
using namespace xyws;
static_assert(detail::calc_frame_header_size(websocket_flags::WS_HAS_MASK, 65536) == 14);
static_assert(detail::calc_frame_header_size(websocket_flags::WS_NONE, 125) == 2);
static_assert(detail::calc_frame_size(websocket_flags::WS_HAS_MASK, 256) == 264);
static_assert(websocket_flags_not_none(websocket_flags::WS_FIN | websocket_flags::WS_OP_TEXT));
int main() {
  try {
    context ctx(0);
    std::puts("device");
    return 0;
  } catch (const error& e) {
    std::printf("error %d\n", e.code());
    return 0;
  }
}
"""


def test_cpp_shim_compiles_links_and_fails_loudly(tmp_path):
    """include/xyws/websocket.hpp (xynet names over the C-ABI) builds with g++
    -std=c++20 against libxyws.so; without a GPU the context throws."""
    src = tmp_path / "shim.cpp"
    src.write_text(SHIM_PROG)
    exe = tmp_path / "shim"
    libdir = os.path.dirname(L.lib_path())
    r = subprocess.run(["g++", "-std=c++20", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                        str(src), "-o", str(exe), "-L", libdir, "-lxyws", f"-Wl,-rpath,{libdir}"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    assert out.stdout.strip() == ("device" if has_gpu else "error -2")
