#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03e_sweep_all.log 2>&1; rc=$?; tail -15 gpurun_out/r03e_sweep_all.log; [ $rc -eq 0 ] || exit $rc
for c in c3 c2 c1 c4; do
  for x in 0 0x1000000; do
    echo "$c xopts=$x $(timeout -k 10 120 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --xopts $x 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' ')" | tee -a gpurun_out/r03e_bench.log
  done
done
