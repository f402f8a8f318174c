#!/bin/bash
cd $GRAFT_REPO_ROOT
true
for c in c3 c2 c1 c4; do
  for x in 0 0x1000000; do
    echo "$c xopts=$x $(timeout -k 10 120 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --xopts $x 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' ')" | tee -a gpurun_out/r03h_bench.log
  done
done
for c in c3 c2 c1 c4; do timeout -k 10 120 python bench.py --config $c --steps 5 --warmup 2 --no-cpu --stats 2>/dev/null | grep '^{"stats"' | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())['stats']; print('$c', {k:v for k,v in d.items() if v and ('sweep' in k or k in ('spins','scan_undecided','dense_passes','runs_without_entry','bad_boundaries','repairs'))})"; done
