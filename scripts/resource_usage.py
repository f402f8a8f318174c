"""Per-kernel register / scratch / occupancy table of one HIP source, from
hipcc's -Rpass-analysis=kernel-resource-usage remarks (gfx950, the build's
flags). Usage: python scripts/resource_usage.py xynet_amd/csrc/xyws_stream.hip [name-filter] [-D...]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from xynet_amd.build import COMMON  # noqa: E402

KEYS = ["VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "SGPRs Spill", "VGPRs Spill",
        "LDS Size [bytes/block]"]


def usage(src, extra=()):
    cmd = ["/opt/rocm/bin/hipcc"] + [f for f in COMMON if f != "-shared"] + list(extra) + [
        "-c", src, "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr[-4000:])
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = {"name": subprocess.run(["c++filt"], input=v, capture_output=True, text=True).stdout.strip()}
            rows.append(cur)
        elif cur is not None and k in KEYS:
            cur[k] = v
    return rows


if __name__ == "__main__":
    src = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else ""
    extra = [a for a in sys.argv[2:] if a.startswith("-")]
    for r in usage(src, extra):
        if flt and flt not in r["name"]:
            continue
        name = re.sub(r"\(anonymous namespace\)::", "", r["name"])
        print(f"{name[:90]:90s} vgpr {r.get('VGPRs','?'):>4} agpr {r.get('AGPRs','?'):>3} "
              f"vspill {r.get('VGPRs Spill','?'):>4} sspill {r.get('SGPRs Spill','?'):>4} "
              f"scratch {r.get('ScratchSize [bytes/lane]','?'):>4} occ {r.get('Occupancy [waves/SIMD]','?')}")
