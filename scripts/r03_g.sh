#!/bin/bash
# Round-3 profile set (TAG r03g): GPU suite, bench lines c3 (full) + c2/c1/c4, c1 forced sweep,
# steady-state kernel traces, PMC traffic (c3, c2, c1, c4), op benches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03g}
step() { local n=$1 s=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $s "$@" > gpurun_out/${T}_$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -2 gpurun_out/${T}_$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for c in c2 c1 c4 c3; do CFG=$c REPS=2 timeout -k 10 400 scripts/abn.sh v1=$PWD/abl/libxyws_v1.so bnd=$PWD/abl/libxyws_bnd.so stride=cur >> gpurun_out/${T}_ab_boundary.log 2>&1 || exit 1; done; cat gpurun_out/${T}_ab_boundary.log
step bench_c3 400 python bench.py --config c3
for c in c2 c1 c4; do step bench_$c 300 python bench.py --config $c --no-ceiling; done
step c1_sweep 200 python bench.py --config c1 --no-cpu --no-ceiling --xopts 0x1000000
for c in c3 c2 c1 c4; do
  step prof_$c 400 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/${T}_prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 30 --warmup 5 --no-cpu --no-ceiling
  python scripts/trace_summary.py --skip 5 gpurun_out/${T}_prof_$c > gpurun_out/${T}_prof_${c}_summary.json
  step pmcf_$c 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $PWD/gpurun_out/${T}_pmc_${c}_fetch -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 3 --no-cpu --no-ceiling
  step pmcw_$c 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $PWD/gpurun_out/${T}_pmc_${c}_write -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 3 --no-cpu --no-ceiling
done
for c in c3 c2; do for op in encode classify reassemble; do step op_${op}_$c 200 python bench.py --config $c --op $op --steps 10 --warmup 2; done; done
step prof_ops_c3 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/${T}_prof_ops_c3 -o run --output-format csv -- python3 bench.py --config c3 --op encode --steps 10 --warmup 2
step prof_rs_c3 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/${T}_prof_rs_c3 -o run --output-format csv -- python3 bench.py --config c3 --op reassemble --steps 5 --warmup 1
step stats_c3 200 python bench.py --config c3 --steps 5 --warmup 3 --no-cpu --no-ceiling --stats
