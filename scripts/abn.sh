#!/bin/bash
# Interleaved A/B of library builds on one box (diagnostic):
#   [CFG=c3] [REPS=4] scripts/abn.sh name=path ...   (path "cur" = the in-tree build)
# prints, per repetition and build, the event-timed ms per decode and parity.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in $(seq ${REPS:-4}); do
  for spec in "$@"; do
    n=${spec%%=*}; lib=${spec#*=}; [ "$lib" = cur ] && lib=$PWD/xynet_amd/libxyws.so
    r=$(XYWS_LIB=$lib timeout -k 10 120 python bench.py --config ${CFG:-c3} --steps ${STEPS:-20} --warmup 3 --no-cpu ${XARGS:-} 2>/dev/null | grep -o '"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' ')
    [ -n "$r" ] || { echo "$n FAILED"; exit 3; }
    echo "$i ${CFG:-c3} $n $r"
  done
done
