#!/bin/bash
cd $GRAFT_REPO_ROOT
for c in c3 c2 c1 c4; do
  for x in 0 0x1000000; do
    echo "$c xopts=$x $(timeout -k 10 120 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --xopts $x 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' ')" | tee -a gpurun_out/r03f_bench.log
  done
done
for c in c3 c2 c1 c4; do timeout -k 10 120 python bench.py --config $c --steps 5 --warmup 2 --no-cpu --stats 2>/dev/null | grep stats | tee -a gpurun_out/r03f_stats.log; done
