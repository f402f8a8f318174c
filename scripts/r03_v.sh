#!/bin/bash
# four 256-thread workgroups per CU (32 KiB segments) vs the geometry choice, c2/c1/c4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
one() { r=$(timeout -k 10 120 python bench.py --config $4 --steps 20 --warmup 3 --no-cpu --no-ceiling $2 2>/dev/null | grep -o '"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*\|"decoder": "[^"]*"' | tr '\n' ' '); [ -n "$r" ] || { echo "$1 FAILED"; exit 3; }; echo "$3 $4 $1 $r"; }
for c in c2 c1 c4; do for i in 1 2; do
  one def "" $i $c || exit 1
  one wg256 "--xopts 0x2000" $i $c || exit 1
  one wg512 "--xopts 0x40000" $i $c || exit 1
done; done 2>&1 | tee gpurun_out/r03v_ab.log
