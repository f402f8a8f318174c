#!/bin/bash
cd $GRAFT_REPO_ROOT
for x in 0x1000000; do
  timeout -k 10 120 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu --xopts $x --stats > gpurun_out/r03l_$x.log 2>&1 || exit 1
  echo "c3 xopts=$x $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r03l_$x.log)"
  grep '"stats"' gpurun_out/r03l_$x.log
done
