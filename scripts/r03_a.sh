#!/bin/bash
# Round-3 baseline (session 2): c3 bench line (copy ceiling + CPU baseline),
# data-path probes (static / steal / dynamic), steady-state kernel trace,
# per-run timeline and phase stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03a}
step() { local n=$1 s=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $s "$@" > gpurun_out/${T}_$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 gpurun_out/${T}_$n.log; [ $rc -eq 0 ] || exit $rc; }
step bench_c3 240 python bench.py --config c3
step probe6 200 scripts/bw_probe6
step prof_c3 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/${T}_prof_c3 -o run --output-format csv -- python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu --no-ceiling
python scripts/trace_summary.py --skip 5 gpurun_out/${T}_prof_c3 > gpurun_out/${T}_prof_c3_summary.json; cat gpurun_out/${T}_prof_c3_summary.json
step tl_c3 200 python scripts/run_timeline.py c3
step stats_c3 200 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu --no-ceiling --stats
