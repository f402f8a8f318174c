#!/bin/bash
# b3 (row-broadcast boundary pre-pass + 2 positions per lane in the stride pass) vs b2; adversarial stride tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "stride_pass_adversarial or dense_frames or fuzz or config_batches or edge_cases" > gpurun_out/r03i_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03i_tests.log; [ $rc -eq 0 ] || exit $rc
for c in c2 c1 c4 c3; do CFG=$c REPS=2 timeout -k 10 400 scripts/abn.sh b2=$PWD/abl/libxyws_b2.so b3=cur >> gpurun_out/r03i_ab.log 2>&1 || exit 1; done; cat gpurun_out/r03i_ab.log
timeout -k 10 200 python bench.py --config c2 --steps 5 --warmup 2 --no-cpu --no-ceiling --stats 2>/dev/null | grep '^{"stats"' > gpurun_out/r03i_stats_c2.log; python3 -c "
import json; d=json.load(open('gpurun_out/r03i_stats_c2.log'))['stats']; print('c2', {k: v for k, v in d.items() if v})"
