#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 100 scripts/bw_probe6 2>&1 | grep -E "static|dynamic|sweep C=2" | tee gpurun_out/r03j_probe6.log
for x in 0 0x10000000 0x20000000 0x30000000 0x1000000; do
  echo "c3 xopts=$x $(timeout -k 10 120 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu --xopts $x 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' ')" | tee -a gpurun_out/r03j_bench.log
done
