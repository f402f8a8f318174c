"""Build the gfx950 shared libraries in-tree with hipcc (no JIT cache).

  xynet_amd/libxyws.so        the decode path (include/xyws.h C-ABI)
  xynet_amd/libxyws_tools.so  synthetic batches + digests (bench/test infra)

Run:  python -m xynet_amd.build   (or __graft_entry__.build())
"""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INC = os.path.join(ROOT, "include")
ARCH = os.environ.get("XYWS_OFFLOAD_ARCH", "gfx950")

# -falign-loops=64: every loop header on a 64-byte boundary (the decoder's
# small-frame loops measured 2-12 % apart between layouts without it)
COMMON = ["--offload-arch=" + ARCH, "-O3", "-falign-loops=64", "-std=c++17", "-fPIC", "-shared", "-Wall",
          "-Wno-unused-function", "-I" + INC, "-I" + CSRC]

TARGETS = {
    "libxyws.so": ["xyws.hip", "xyws_stream.hip", "xyws_frames.hip", "xyws_arena.hip", "xyws_shard.hip"],
    "libxyws_tools.so": ["xyws_tools.hip"],
}
DEPS = ["xyws_device.h", "xyws_stream.h", "xyws_ctx.h", "xyws_lattice.h"]


def _stale(out, srcs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = [os.path.join(CSRC, s) for s in srcs + DEPS] + [
        os.path.join(INC, "xyws.h"), os.path.join(INC, "xyws_synth.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


OBJ = os.path.join(PKG, ".build")  # per-source objects (git- and gpurun-ignored)


def _run(cmd, what, verbose):
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {what}:\n{r.stdout}\n{r.stderr}")
    if verbose and r.stderr.strip():
        print(r.stderr)


def build(force=False, verbose=False, extra=None):
    """Each source compiles to its own object in parallel (the stream decoder
    alone takes about a minute), then one hipcc link per library."""
    from concurrent.futures import ThreadPoolExecutor
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    os.makedirs(OBJ, exist_ok=True)
    cflags = [f for f in COMMON if f != "-shared"] + (extra or [])
    jobs = []
    for name, srcs in TARGETS.items():
        out = os.path.join(PKG, name)
        if not force and not _stale(out, srcs):
            continue
        objs = [os.path.join(OBJ, os.path.splitext(s)[0] + ".o") for s in srcs]
        jobs.append((name, out, srcs, objs))
    compile_cmds = [([hipcc] + cflags + ["-c", os.path.join(CSRC, s), "-o", o], s)
                    for _, _, srcs, objs in jobs for s, o in zip(srcs, objs)]
    with ThreadPoolExecutor(max_workers=min(8, max(1, len(compile_cmds)))) as ex:
        list(ex.map(lambda c: _run(c[0], c[1], verbose), compile_cmds))
    for name, out, _, objs in jobs:
        _run([hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC"] + objs + ["-o", out], name, verbose)
    build_cpp_tests(hipcc, force=force, verbose=verbose)
    return [os.path.join(PKG, n) for n in TARGETS]


# C++ callers of the header-only shim (include/xyws/websocket.hpp) and of the
# C-ABI (the loopback echo harness), run by the GPU tests: linked against the in-tree libxyws.so (rpath), built here so the
# binary travels to the GPU box with the tree. They are host code only (the
# kernels are libxyws.so's), so g++ builds them, with the HIP runtime API
# headers where they call it (hipcc's device pass crashed on the shim's
# std::views::join overload: clang 22, ROCm 7.2).
CPP_TESTS = {"tests/cpp/test_shim": "tests/cpp/test_shim.cpp", "tests/cpp/test_compat": "tests/cpp/test_compat.cpp",
             "examples/echo_loopback": "examples/echo_loopback.cpp"}


def build_cpp_tests(hipcc, force=False, verbose=False):
    for out, src in CPP_TESTS.items():
        out, src = os.path.join(ROOT, out), os.path.join(ROOT, src)
        deps = [src, os.path.join(INC, "xyws.h"), os.path.join(INC, "xyws", "websocket.hpp"),
                os.path.join(PKG, "libxyws.so")]
        if not force and os.path.exists(out) and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps):
            continue
        rpath = os.path.relpath(PKG, os.path.dirname(out))
        rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
        cmd = [os.environ.get("CXX", "g++"), "-std=c++20", "-O2", "-Wall", "-I" + INC, "-I" + rocm + "/include",
               "-D__HIP_PLATFORM_AMD__", src, "-o", out, "-L" + PKG, "-lxyws", "-L" + rocm + "/lib", "-lamdhip64",
               "-Wl,-rpath,$ORIGIN/" + rpath + ":" + rocm + "/lib"]
        if verbose:
            print(" ".join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {out}:\n{r.stdout}\n{r.stderr}")


if __name__ == "__main__":
    print("\n".join(build(force="--force" in sys.argv, verbose=True)))
