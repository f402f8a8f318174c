#!/usr/bin/env python3
"""Per-kernel dispatch durations from rocprofv3 kernel traces (diagnostic).

usage: trace_summary.py [--skip N] DIR...
For every decoder kernel (k_stream_*, k_enc_*, k_gather, k_classify, k_rs_*,
k_utf8, k_unmask_*): dispatch count, mean / median / min / max in us, over all
dispatches and over the steady state (the first N dispatches of each kernel
dropped: bench.py's warm-up steps, whose first call also pays code-object load
and cold caches). Prints one JSON object per DIR.
"""
import csv
import glob
import json
import statistics
import sys

KERNELS = ("k_stream_", "k_enc_", "k_gather", "k_classify", "k_rs_", "k_utf8", "k_unmask_", "k_parse_", "k_scan_")


def short(name):
    for k in KERNELS:
        if k in name:
            return k + name.split(k)[1].split("<")[0].split("(")[0]
    return None


def stats(v):
    return {"n": len(v), "mean": round(statistics.mean(v), 2), "median": round(statistics.median(v), 2),
            "min": round(min(v), 2), "max": round(max(v), 2)}


def main():
    args = sys.argv[1:]
    skip = 0
    if args[:1] == ["--skip"]:
        skip, args = int(args[1]), args[2:]
    for d in args:
        f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
        if not f:
            print(json.dumps({"dir": d, "error": "no trace"}))
            continue
        rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"]))
        out = {}
        for r in rows:
            k = short(r["Kernel_Name"])
            if k:
                out.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
        res = {"dir": d, "skip": skip}
        for k, v in out.items():
            res[k] = {"all": stats(v)}
            if len(v) > skip:
                res[k]["steady"] = stats(v[skip:])
        print(json.dumps(res))


if __name__ == "__main__":
    main()
