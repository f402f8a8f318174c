"""Overlap of H2D copies, decode kernels and D2H copies in a host-path run.

Reads a rocprofv3 output directory holding *kernel_trace.csv and
*memory_copy_trace.csv (rocprofv3 --kernel-trace --memory-copy-trace) and
prints one JSON object: the busy time of each engine class (union of its
intervals), the wall span, and how much of each class's busy time overlaps the
others' -- the per-stream overlap timeline of bench.py --host-path in numbers.

  python scripts/overlap_summary.py DIR [--skip-ms 0]
"""
import csv
import glob
import json
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def total(iv):
    return sum(b - a for a, b in iv)


def intersect(x, y):
    i = j = 0
    out = []
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            out.append([a, b])
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return out


def main():
    d = sys.argv[1]
    skip = float(sys.argv[sys.argv.index("--skip-ms") + 1]) * 1e6 if "--skip-ms" in sys.argv else 0.0
    kf = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    mf = glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True)
    assert kf and mf, "need kernel and memory-copy traces"
    cls = {"kernel": [], "h2d": [], "d2h": [], "d2d": []}
    for r in csv.DictReader(open(kf[0])):
        if "k_stream" in r["Kernel_Name"] or "k_unmask" in r["Kernel_Name"]:
            cls["kernel"].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for r in csv.DictReader(open(mf[0])):
        kind = " ".join(str(v) for k, v in r.items() if k in ("Direction", "Operation", "Kind")).upper()
        key = "h2d" if "HOST_TO_DEVICE" in kind else "d2h" if "DEVICE_TO_HOST" in kind else "d2d"
        cls[key].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    t0 = min(a for v in cls.values() for a, _ in v) + skip
    cls = {k: union([(max(a, t0), b) for a, b in v if b > t0]) for k, v in cls.items()}
    span = max(b for v in cls.values() for _, b in v) - t0
    out = {"span_ms": span / 1e6}
    for k, v in cls.items():
        if not v:
            continue
        others = union([iv for k2, v2 in cls.items() if k2 != k for iv in v2])
        out[k] = {"n": len(v), "busy_ms": total(v) / 1e6, "busy_frac_of_span": total(v) / span,
                  "overlapped_frac": total(intersect(v, others)) / max(total(v), 1)}
    copies = union(cls["h2d"] + cls["d2h"])
    out["kernel_hidden_under_copies_frac"] = total(intersect(cls["kernel"], copies)) / max(total(cls["kernel"]), 1)
    out["h2d_d2h_concurrent_ms"] = total(intersect(cls["h2d"], cls["d2h"])) / 1e6
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
