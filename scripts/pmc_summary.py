#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes of the bench into profiles/pmc_traffic.json.

HBM traffic per launch of the decoder kernel the timed steps ran (k_stream_lattice or k_stream_runs), per MI355X_MICROARCH.md §HBM: gfx950's
FETCH_SIZE reports half the bytes of wide coalesced streaming reads (doubled
here); WRITE_SIZE reads the bytes exactly for 16-B-per-lane stores. Both
counters are in KiB. Usage: pmc_summary.py FETCH_DIR WRITE_DIR KEY PROFILE [OUT]
KEY is "<config>:<mode>"; the record is stamped with the decoder sources' hash
(bench.source_hash) so bench.py only reports traffic measured on this kernel.
"""
import csv
import glob
import json
import os
import sys


def per_launch(d, counter, kernel=None):
    """Average counter value per launch of `kernel` (a name substring); by
    default the decoder kernel (k_stream_lattice / k_stream_runs /
    k_stream_lattice) of the last dispatches, i.e. the one the timed steps ran
    (the decoder choice serves the first calls, before the first one has
    finished, with the run decoder); after a lattice launch the run decoder
    that follows it reads the redirect record and exits: the lattice's counts."""
    names = ("k_stream_lattice", "k_stream_runs")
    vals, last, prev = {}, None, None
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows = list(csv.DictReader(open(f)))
        if rows and "Dispatch_Id" in rows[0]:
            rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        for r in rows:
            name = r["Kernel_Name"]
            hit = (kernel in name) if kernel else any(n in name for n in names)
            if hit and r["Counter_Name"] == counter:
                k = kernel or next(n for n in names if n in name)
                redirect = prev == "k_stream_lattice" and k == "k_stream_runs"  # (the lattice's hand-over check)
                prev = k
                if redirect:
                    continue
                vals.setdefault(k, []).append(float(r["Counter_Value"]))
                last = k
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel or 'the decoder kernels'} under {d}")
    k = last  # (the timed steps are the last dispatches)
    v = vals[k]
    return sum(v) / len(v), len(v), k


def source_hash():
    import hashlib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    h = hashlib.sha256()
    for f in ("xyws_stream.hip", "xyws_device.h", "xyws_stream.h", "xyws.hip", "xyws_lattice.h"):
        with open(os.path.join(root, "xynet_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def main():
    fdir, wdir, key, profile = sys.argv[1:5]
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    fk, nf, kf = per_launch(fdir, "FETCH_SIZE")
    wk, nw, kw = per_launch(wdir, "WRITE_SIZE")
    assert kf == kw, (kf, kw)
    rec = {
        "kernel": kf,
        "fetch_size_kib_raw": fk, "write_size_kib": wk, "launches": [nf, nw],
        "hbm_read_bytes_per_launch": int(fk * 2 * 1024),
        "hbm_write_bytes_per_launch": int(wk * 1024),
        "hbm_bytes_per_launch": int(fk * 2 * 1024 + wk * 1024),
        "correction": "FETCH_SIZE x2 (gfx950 streaming-read undercount), KiB -> bytes",
        "src_sha": os.environ.get("PMC_SRC_SHA") or source_hash(),  # (override: the profiled tree's hash)
        "profile": profile,
    }
    data = json.load(open(out)) if os.path.exists(out) else {}
    data[key] = rec
    json.dump(data, open(out, "w"), indent=1)
    print(json.dumps({key: rec}))


if __name__ == "__main__":
    main()
