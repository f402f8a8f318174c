"""Top kernels of a rocprofv3 --stats CSV directory: average us, calls, name.
usage: kstats.py DIR [N]"""
import csv
import os
import sys


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    rows = list(csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))))
    for r in rows[:n]:
        print("%9.2f %5s %s" % (float(r["AverageNs"]) / 1000, r["Calls"], r["Name"][:100]))


if __name__ == "__main__":
    main()
