#!/bin/bash
# split-role sweep: parity first, then c3 timing (sweep vs sweep+loadwait vs runs) and the stats split
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sweep.py > gpurun_out/r03m_tests.log 2>&1 || { tail -30 gpurun_out/r03m_tests.log; exit 1; }
tail -2 gpurun_out/r03m_tests.log
for x in 0x1000000 0x41000000 0; do
  echo "c3 xopts=$x $(timeout -k 10 120 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu --xopts $x 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' ')"
done
timeout -k 10 120 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu --xopts 0x1000000 --stats > gpurun_out/r03m_stats.log 2>&1 || exit 1
grep '"stats"' gpurun_out/r03m_stats.log
