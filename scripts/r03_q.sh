#!/bin/bash
# lattice passes in the run decoder (c1/c2), k_gather fast path only for tiles of <= 3 items
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03q_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03q_tests.log; [ $rc -eq 0 ] || exit $rc
one() { r=$(XYWS_LIB=$2 timeout -k 10 120 python bench.py --config $5 --steps 20 --warmup 3 --no-cpu --no-ceiling $3 2>/dev/null | grep -o '"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' '); [ -n "$r" ] || { echo "$1 FAILED"; exit 3; }; echo "$4 $5 $1 $r"; }
for c in c2 c1 c4; do for i in 1 2; do
  one b2 $PWD/abl/libxyws_b2.so "" $i $c || exit 1
  one new $PWD/xynet_amd/libxyws.so "" $i $c || exit 1
  one nolat $PWD/xynet_amd/libxyws.so "--xopts 0x200000" $i $c || exit 1
done; done 2>&1 | tee gpurun_out/r03q_ab.log
for c in c3 c2 c1; do for op in encode; do timeout -k 10 200 python bench.py --config $c --op $op --steps 10 --warmup 2 2>/dev/null | tee -a gpurun_out/r03q_ops.log | grep -o '"op": "[a-z]*"\|"value": [0-9.]*\|"frac": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' '; echo " $c"; done; done
timeout -k 10 200 python bench.py --config c2 --no-cpu --no-ceiling --steps 5 --warmup 3 --stats > gpurun_out/r03q_stats_c2.log 2>&1 || exit 1
grep -o '"stats".*' gpurun_out/r03q_stats_c2.log | cut -c1-2500
