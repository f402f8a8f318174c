#!/bin/bash
# stride pass 4 positions/lane; lattice entry from the previous call's frame size; run-decoder geometry choice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "lattice_entry or stride or config_batches" > gpurun_out/r03u_tests1.log 2>&1; rc=$?; tail -3 gpurun_out/r03u_tests1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03u_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03u_tests.log; [ $rc -eq 0 ] || exit $rc
one() { r=$(XYWS_LIB=$2 timeout -k 10 120 python bench.py --config $5 --steps 20 --warmup 3 --no-cpu --no-ceiling $3 2>/dev/null | grep -o '"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' '); [ -n "$r" ] || { echo "$1 FAILED"; exit 3; }; echo "$4 $5 $1 $r"; }
for c in c2 c1 c4; do for i in 1 2; do
  one b3 $PWD/abl/libxyws_b3.so "" $i $c || exit 1
  one new $PWD/xynet_amd/libxyws.so "" $i $c || exit 1
  one nolatentry $PWD/xynet_amd/libxyws.so "--xopts 0x4000" $i $c || exit 1
done; done 2>&1 | tee gpurun_out/r03u_ab.log
timeout -k 10 200 python bench.py --config c2 --no-cpu --no-ceiling --steps 5 --warmup 3 --stats > gpurun_out/r03u_stats_c2.log 2>&1 || exit 1
grep -o '"stats".*' gpurun_out/r03u_stats_c2.log | cut -c1-2500
