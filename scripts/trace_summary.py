#!/usr/bin/env python3
"""Mean duration per decoder kernel from rocprofv3 kernel traces: trace_summary.py DIR..."""
import csv, glob, statistics, sys
for d in sys.argv[1:]:
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
    if not f:
        print(d, "no trace"); continue
    rows = list(csv.DictReader(open(f[0])))
    out = {}
    for r in rows:
        n = r["Kernel_Name"]
        if "k_stream" not in n: continue
        k = n.split("k_stream_")[1].split("<")[0].split("(")[0]
        out.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    print(d, {k: (round(statistics.mean(v), 2), len(v)) for k, v in out.items()})
