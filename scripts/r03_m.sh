#!/bin/bash
# sweep look-ahead (next segment's list built during the stores) + k_utf8 chunk loads: full GPU suite, c3 A/B, reassemble benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03m_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03m_tests.log; [ $rc -eq 0 ] || exit $rc
CFG=c3 REPS=3 bash scripts/abn.sh b2=$PWD/abl/libxyws_b2.so new=cur 2>&1 | tee gpurun_out/r03m_ab_c3.log || exit 1
CFG=c1 REPS=2 bash scripts/abn.sh b2=$PWD/abl/libxyws_b2.so new=cur 2>&1 | tee gpurun_out/r03m_ab_c1.log || exit 1
for c in c1 c2 c3; do timeout -k 10 200 python bench.py --config $c --op reassemble --steps 10 --warmup 2 2>/dev/null | tee -a gpurun_out/r03m_ops.log | grep -o '"value": [0-9.]*\|"frac": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' '; echo " $c"; done
