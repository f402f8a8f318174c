#!/bin/bash
# zero_now fix: the concurrent-decode test 5 times, then the whole GPU suite, then the c3 line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for i in 1 2 3 4 5; do
  timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -k "concurrent_decodes" > gpurun_out/r03f_conc_$i.log 2>&1; echo "conc $i rc=$? $(tail -1 gpurun_out/r03f_conc_$i.log)"
done
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03f_gpu_tests.log 2>&1; rc=$?; tail -5 gpurun_out/r03f_gpu_tests.log
timeout -k 10 300 python bench.py --config c3 > gpurun_out/r03f_bench_c3.log 2>&1; tail -1 gpurun_out/r03f_bench_c3.log | cut -c1-400
exit $rc
