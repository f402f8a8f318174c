#!/bin/bash
# Per-run timelines (scripts/run_timeline.py) of library variants (diagnostic):
#   scripts/tl_variants.sh CFG NAME...   (cur = the in-tree library)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cfg=$1; shift
for name in "$@"; do
  lib=$PWD/exp/libxyws_$name.so; [ "$name" = cur ] && lib=$PWD/xynet_amd/libxyws.so
  echo "$name $(XYWS_LIB=$lib timeout -k 10 120 python scripts/run_timeline.py $cfg 2>/dev/null | grep '^{' | python3 -c '
import json,sys
d=json.loads(sys.stdin.read()); d.pop("latest_runs"); d.pop("end_us_by_run_mod8"); print(json.dumps(d))')"
done
