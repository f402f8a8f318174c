#!/bin/bash
# run-decoder geometry choice (512-thread workgroups after regular frames < 2 KiB); RUNS_NOWAIT experiment; stride-pass timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03t_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03t_tests.log; [ $rc -eq 0 ] || exit $rc
one() { r=$(timeout -k 10 120 python bench.py --config $4 --steps 20 --warmup 3 --no-cpu --no-ceiling $2 2>/dev/null | grep -o '"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*\|"decoder": "[^"]*"' | tr '\n' ' '); [ -n "$r" ] || { echo "$1 FAILED"; exit 3; }; echo "$3 $4 $1 $r"; }
for c in c2 c1; do for i in 1 2; do
  one def "" $i $c || exit 1
  one nowait "--xopts 0x10000" $i $c || exit 1
  one wg1024 "--xopts 0x8000" $i $c || exit 1
done; done 2>&1 | tee gpurun_out/r03t_ab.log
for x in "" "--xopts 0x8000"; do timeout -k 10 200 python bench.py --config c2 --no-cpu --no-ceiling --steps 5 --warmup 3 --stats $x > gpurun_out/r03t_stats_c2.log 2>&1 || exit 1
grep -o '"stats".*' gpurun_out/r03t_stats_c2.log | cut -c1-2500; done
