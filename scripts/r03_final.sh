#!/bin/bash
# Round-3 profile set (TAG r03x) on the committed sources: GPU suite + smoke, bench lines,
# steady-state kernel traces, PMC traffic per config, op benches, compatibility-path latency
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03x}
step() { local n=$1 s=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $s "$@" > gpurun_out/${T}_$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -1 gpurun_out/${T}_$n.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc; }
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c3 400 python bench.py --config c3
for c in c2 c1 c4; do step bench_$c 300 python bench.py --config $c --no-ceiling; done
for c in c3 c2 c1 c4; do
  step prof_$c 400 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/${T}_prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 30 --warmup 5 --no-cpu --no-ceiling
  python scripts/trace_summary.py --skip 5 gpurun_out/${T}_prof_$c > gpurun_out/${T}_prof_${c}_summary.json
  step pmcf_$c 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $PWD/gpurun_out/${T}_pmc_${c}_fetch -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 3 --no-cpu --no-ceiling
  step pmcw_$c 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $PWD/gpurun_out/${T}_pmc_${c}_write -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 3 --no-cpu --no-ceiling
done
step compat 120 tests/cpp/test_compat --latency
step host_c3 400 python bench.py --config c3 --no-cpu --no-ceiling --host-path --steps 5
for c in c3 c2; do for op in encode classify reassemble; do
  step op_${op}_$c 300 python bench.py --config $c --op $op --no-cpu --no-ceiling
done; done
step prof_ops_c3 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/${T}_prof_ops_c3 -o run --output-format csv -- python3 bench.py --config c3 --op encode --no-cpu --no-ceiling --steps 10 --warmup 2
for c in 4096 65536; do step echo_$c 120 examples/echo_loopback --frames 200000 --chunk $c; done
step echo_ping 120 examples/echo_loopback --frames 200000 --chunk 65536 --ping-every 10
step echo_125 120 examples/echo_loopback --frames 400000 --max-len 125 --chunk 65536
step echo_prof 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/${T}_echo_prof -o run --output-format csv -- examples/echo_loopback --frames 200000 --chunk 65536
for sz in 262144 4194304; do for o in 0 0x8000; do
  timeout -k 10 120 python scripts/small_batch_stats.py $sz $o || exit 1
done; done > gpurun_out/${T}_small_stats.jsonl 2>&1
echo "== small stats"; cut -c1-200 gpurun_out/${T}_small_stats.jsonl
