#!/bin/bash
# rocprofv3 kernel trace of bench.py c3 for each build (cur = the in-tree library): per-kernel durations
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
tag=${TAG:-ab}
for rev in "$@"; do
  lib=$PWD/exp/libxyws_$rev.so; [ "$rev" = cur ] && lib=$PWD/xynet_amd/libxyws.so
  XYWS_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/${tag}_prof_$rev -o run --output-format csv -- python3 bench.py --config ${CFG:-c3} --steps 10 --warmup 2 --no-cpu > gpurun_out/${tag}_prof_$rev.log 2>&1 || exit 1
done
