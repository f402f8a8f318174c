#!/bin/bash
# A/B: v1 (validate fix) vs b2 (boundary pre-XOR with row classes first + stride pass + inline finisher);
# c2 stats with b2 (does the stride pass take the dense segments?)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modes.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03h_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03h_tests.log; [ $rc -eq 0 ] || exit $rc
for c in c1 c2 c3 c4; do CFG=$c REPS=2 timeout -k 10 400 scripts/abn.sh v1=$PWD/abl/libxyws_v1.so b2=cur >> gpurun_out/r03h_ab.log 2>&1 || exit 1; done; cat gpurun_out/r03h_ab.log
for c in c2 c1; do timeout -k 10 200 python bench.py --config $c --steps 5 --warmup 2 --no-cpu --no-ceiling --stats 2>/dev/null | grep '^{"stats"' > gpurun_out/r03h_stats_$c.log; python3 -c "
import json; d=json.load(open('gpurun_out/r03h_stats_$c.log'))['stats']; print('$c', {k: v for k, v in d.items() if v})"; done
