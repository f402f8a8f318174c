set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
T=r05b
step() { local n=$1 s=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $s "$@" > gpurun_out/${T}_$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 gpurun_out/${T}_$n.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lattice.py tests/test_gpu_choice.py tests/test_gpu_graph.py tests/test_gpu_parity.py -k "lattice or choice or graph or captured or replay or lat or bench_path or config_batches"
for c in c3 c2 c1 c4; do step bench_$c 300 python bench.py --config $c --no-cpu --no-ceiling; done
step choice 200 python scripts/choice_trace.py c3,c3,c4,c4,c4,c3,c3
step prof 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/${T}_prof -o run --output-format csv -- python3 scripts/choice_trace.py c3,c3,c4,c4,c4,c2,c2,c2
echo done
