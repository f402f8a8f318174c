#!/bin/bash
# sweep decoder timing split on c3 (stats build) + headline A/B + shim compat program
cd $GRAFT_REPO_ROOT
timeout -k 10 60 tests/cpp/test_compat > gpurun_out/r03k_compat.log 2>&1 || exit 1
timeout -k 10 60 tests/cpp/test_compat --latency >> gpurun_out/r03k_compat.log 2>&1 || exit 1
cat gpurun_out/r03k_compat.log
for x in 0x1000000 0x11000000; do
  timeout -k 10 120 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu --xopts $x --stats > gpurun_out/r03k_$x.log 2>&1 || exit 1
  echo "c3 xopts=$x $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r03k_$x.log)"
  grep '"stats"' gpurun_out/r03k_$x.log
done
echo "runs $(timeout -k 10 120 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')"
