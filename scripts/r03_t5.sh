#!/bin/bash
cd $GRAFT_REPO_ROOT
for c in c3 c2; do timeout -k 10 120 python bench.py --config $c --steps 5 --warmup 2 --no-cpu --stats 2>/dev/null | grep '^{"stats"' | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())['stats']; print('$c', {k:v for k,v in d.items() if v and ('sweep' in k or k in ('spins','scan_undecided','dense_passes','runs_without_entry'))})"; done
