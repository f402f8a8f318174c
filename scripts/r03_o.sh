#!/bin/bash
# k_gather fast path (lane-shuffled second line) + look-ahead variants: full GPU suite, c3 variants, op benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03o_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03o_tests.log; [ $rc -eq 0 ] || exit $rc
one() { r=$(XYWS_LIB=$2 timeout -k 10 120 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu --no-ceiling $3 2>/dev/null | grep -o '"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' '); [ -n "$r" ] || { echo "$1 FAILED"; exit 3; }; echo "$4 c3 $1 $r"; }
for i in 1 2; do
  one b2 $PWD/abl/libxyws_b2.so "" $i || exit 1
  one new $PWD/xynet_amd/libxyws.so "" $i || exit 1
  one noahead $PWD/xynet_amd/libxyws.so "--xopts 0x200000" $i || exit 1
  one loadwait $PWD/xynet_amd/libxyws.so "--xopts 0x40000000" $i || exit 1
done 2>&1 | tee gpurun_out/r03o_c3var.log
for c in c3 c2 c1; do for op in encode reassemble; do timeout -k 10 200 python bench.py --config $c --op $op --steps 10 --warmup 2 2>/dev/null | tee -a gpurun_out/r03o_ops.log | grep -o '"op": "[a-z]*"\|"value": [0-9.]*\|"frac": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' '; echo " $c"; done; done
