#!/usr/bin/env python3
"""Memory operations, waits and barriers of one kernel in hipcc -S output,
with their source locations (diagnostic: find loads whose registers are
spilled or waited for at once).

usage: isa_marks.py FILE.s KERNEL_SUBSTRING [--calls]
Compile first with: hipcc ... --offload-device-only -S -gline-tables-only.
"""
import re
import sys


def main():
    path, want = sys.argv[1], sys.argv[2]
    s = open(path).read().split("\n")
    files = {}
    for l in s:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s*(?:"([^"]*)")?', l)
        if m:
            files[int(m.group(1))] = (m.group(3) or m.group(2)).split("/")[-1]
    start = None
    for i, l in enumerate(s):
        if re.match(r"^_Z\S*:", l) and want in l:
            start = i
            break
    if start is None:
        sys.exit("kernel not found")
    end = start
    while not s[end].startswith(".Lfunc_end"):
        end += 1
    loc = None
    pat = re.compile(r"s_waitcnt vmcnt\(|global_atomic|scratch_|buffer_load|buffer_store|global_load|global_store|s_barrier|s_swappc|s_setpc")
    for i in range(start, end):
        l = s[i]
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            loc = f"{files.get(int(m.group(1)), '?')}:{m.group(2)}"
        if pat.search(l) or re.match(r"^\.LBB\S*:", l):
            print(f"{i - start:6d} {loc or '-':28s} {l.strip()[:80]}")


if __name__ == "__main__":
    main()
