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

COMMON = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
          "-Wno-unused-function", "-I" + INC, "-I" + CSRC]

TARGETS = {
    "libxyws.so": ["xyws.hip", "xyws_stream.hip"],
    "libxyws_tools.so": ["xyws_tools.hip"],
}
DEPS = ["xyws_device.h", "xyws_stream.h"]


def _stale(out, srcs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = [os.path.join(CSRC, s) for s in srcs + DEPS] + [
        os.path.join(INC, "xyws.h"), os.path.join(INC, "xyws_synth.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False, extra=None):
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    for name, srcs in TARGETS.items():
        out = os.path.join(PKG, name)
        if not force and not _stale(out, srcs):
            continue
        cmd = [hipcc] + COMMON + (extra or []) + [os.path.join(CSRC, s) for s in srcs] + ["-o", out]
        if verbose:
            print(" ".join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {name}:\n{r.stdout}\n{r.stderr}")
        if verbose and r.stderr.strip():
            print(r.stderr)
    return [os.path.join(PKG, n) for n in TARGETS]


if __name__ == "__main__":
    print("\n".join(build(force="--force" in sys.argv, verbose=True)))
