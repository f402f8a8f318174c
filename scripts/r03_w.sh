#!/bin/bash
# Loopback echo harness (examples/echo_loopback) + device-side partial parser
# result: GPU tests for both, echo throughput at several client write sizes,
# kernel stats of one echo run
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03w}
step() { local n=$1 s=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $s "$@" > gpurun_out/${T}_$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -1 gpurun_out/${T}_$n.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step tests 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_echo_loopback.py tests/test_gpu_modes.py tests/test_cpp_shim.py
for c in 4096 65536 1048576; do
  step echo_$c 120 examples/echo_loopback --frames 200000 --chunk $c
done
step echo_ping 120 examples/echo_loopback --frames 200000 --chunk 65536 --ping-every 10
step echo_125 120 examples/echo_loopback --frames 400000 --max-len 125 --chunk 65536
step echo_prof 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/${T}_echo_prof -o run --output-format csv -- examples/echo_loopback --frames 200000 --chunk 65536
step compat 120 tests/cpp/test_compat --latency
step host_tl 300 rocprofv3 --kernel-trace --memory-copy-trace -d $PWD/gpurun_out/${T}_host_tl -o run --output-format csv -- python3 bench.py --config c3 --no-cpu --no-ceiling --host-path --steps 3 --warmup 1
python scripts/overlap_summary.py gpurun_out/${T}_host_tl > gpurun_out/${T}_host_overlap.json 2>&1; cat gpurun_out/${T}_host_overlap.json | head -40
