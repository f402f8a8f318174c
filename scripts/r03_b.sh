#!/bin/bash
# c3: run decoder vs sweep decoder (segment claiming) on one box, with the sweep's timing split
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for x in 0 0x1000000 0x41000000 0 0x1000000; do
  echo "c3 xopts=$x $(timeout -k 10 120 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu --no-ceiling --xopts $x 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' ')" | tee -a gpurun_out/r03b_ab.log
done
timeout -k 10 120 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu --no-ceiling --stats --xopts 0x1000000 > gpurun_out/r03b_sweep_stats.log 2>&1 || exit 1
grep '"stats"' gpurun_out/r03b_sweep_stats.log
timeout -k 10 120 python scripts/run_timeline.py c3 0x1000000 > gpurun_out/r03b_sweep_tl.log 2>&1; tail -c 1500 gpurun_out/r03b_sweep_tl.log
