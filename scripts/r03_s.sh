#!/bin/bash
# WG512 (two 512-thread workgroups per CU, 64 KiB segments) vs default on the run decoder configs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
one() { r=$(timeout -k 10 120 python bench.py --config $4 --steps 20 --warmup 3 --no-cpu --no-ceiling $2 2>/dev/null | grep -o '"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' '); [ -n "$r" ] || { echo "$1 FAILED"; exit 3; }; echo "$3 $4 $1 $r"; }
for c in c2 c1 c4; do for i in 1 2; do
  one def "" $i $c || exit 1
  one wg512 "--xopts 0x40000" $i $c || exit 1
done; done 2>&1 | tee gpurun_out/r03s_wg512.log
timeout -k 10 200 python bench.py --config c2 --no-cpu --no-ceiling --steps 5 --warmup 3 --stats --xopts 0x40000 > gpurun_out/r03s_stats_c2_wg512.log 2>&1 || exit 1
grep -o '"stats".*' gpurun_out/r03s_stats_c2_wg512.log | cut -c1-2500
