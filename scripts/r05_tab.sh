set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r05g}
step() { local n=$1 s=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $s "$@" > gpurun_out/${T}_$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 gpurun_out/${T}_$n.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_choice.py -k "tab or choice or bench_path"
step bench_c4 300 python bench.py --config c4 --no-cpu --no-ceiling
step prof 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/${T}_prof -o run --output-format csv -- python3 bench.py --config c4 --steps 20 --warmup 5 --no-cpu --no-ceiling
python scripts/trace_summary.py --skip 5 gpurun_out/${T}_prof > gpurun_out/${T}_prof_summary.json; cat gpurun_out/${T}_prof_summary.json
echo done
