#!/bin/bash
# look-ahead loads at the loop top (ahead of the data loads) + wave-wide boundary-chunk lookup: full GPU suite, A/B c3 c2 c1, sweep stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03n_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r03n_tests.log; [ $rc -eq 0 ] || exit $rc
for c in c3 c2 c1; do CFG=$c REPS=2 bash scripts/abn.sh b2=$PWD/abl/libxyws_b2.so new=cur 2>&1 | tee -a gpurun_out/r03n_ab.log || exit 1; done
timeout -k 10 200 python bench.py --config c3 --no-cpu --steps 5 --warmup 3 --stats > gpurun_out/r03n_stats_c3.log 2>&1 || exit 1
grep -o '"stats".*' gpurun_out/r03n_stats_c3.log | cut -c1-2500
