#!/bin/bash
# decoder choice: policy test, sweep tests, all configs with the default choice vs forced runs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread -k "decoder_choice" > gpurun_out/r03d_policy.log 2>&1; rc=$?; tail -15 gpurun_out/r03d_policy.log; [ $rc -eq 0 ] || exit $rc
for c in c3 c2 c1 c4; do for x in 0 0x80000000; do
  echo "$c xopts=$x $(timeout -k 10 120 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --no-ceiling --xopts $x 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' ')" | tee -a gpurun_out/r03d_ab.log
done; done
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03d_gpu_tests.log 2>&1; rc=$?; tail -5 gpurun_out/r03d_gpu_tests.log; exit $rc
