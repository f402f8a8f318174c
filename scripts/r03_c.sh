#!/bin/bash
# sweep parity + c1/c2/c4 A/B (run vs sweep vs sweep+loadwait); new gather: frames tests + op benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_frames.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03c_frames.log 2>&1; rc=$?; tail -3 gpurun_out/r03c_frames.log; [ $rc -eq 0 ] || exit $rc
for c in c3 c2; do for op in encode classify reassemble; do
  timeout -k 10 120 python bench.py --config $c --op $op --steps 10 --warmup 2 2>/dev/null | tee -a gpurun_out/r03c_ops.log | grep -o '"op": "[a-z]*"\|"value": [0-9.]*\|"frac": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' '; echo " $c"
done; done
for c in c2 c1 c4; do for x in 0 0x1000000 0x41000000; do
  echo "$c xopts=$x $(timeout -k 10 120 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --no-ceiling --xopts $x 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' ')" | tee -a gpurun_out/r03c_ab.log
done; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_sweep.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03c_sweep_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03c_sweep_tests.log; exit $rc
