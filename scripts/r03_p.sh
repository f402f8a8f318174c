#!/bin/bash
# look-ahead removed (prediction at the loop top kept); k_gather second lines issued up front; k_utf8 staged in LDS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03p_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03p_tests.log; [ $rc -eq 0 ] || exit $rc
for c in c3 c2; do CFG=$c REPS=2 bash scripts/abn.sh b2=$PWD/abl/libxyws_b2.so new=cur 2>&1 | tee -a gpurun_out/r03p_ab.log || exit 1; done
for c in c3 c2 c1; do for op in encode reassemble; do timeout -k 10 200 python bench.py --config $c --op $op --steps 10 --warmup 2 2>/dev/null | tee -a gpurun_out/r03p_ops.log | grep -o '"op": "[a-z]*"\|"value": [0-9.]*\|"frac": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' '; echo " $c"; done; done
timeout -k 10 200 python bench.py --config c2 --no-cpu --no-ceiling --steps 5 --warmup 3 --stats > gpurun_out/r03p_stats_c2.log 2>&1 || exit 1
grep -o '"stats".*' gpurun_out/r03p_stats_c2.log | cut -c1-2500
