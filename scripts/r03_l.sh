#!/bin/bash
# k_unmask_range (8 loads in flight per lane) + tile-mapped k_utf8: tests, copy ceiling, op benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_frames.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "unmask or reassemble or encode or echo or compat or mask" > gpurun_out/r03l_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r03l_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_cpp_shim.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03l_shim.log 2>&1; rc=$?; tail -1 gpurun_out/r03l_shim.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --config c3 --no-cpu --steps 20 --warmup 5 > gpurun_out/r03l_c3.log 2>&1 || exit 1
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/r03l_c3.log') if l.startswith('{\"metric')][-1]); print(d['ms_per_step'], d['roofline']['copy_ceiling'])"
for c in c3 c1 c2; do for op in reassemble encode; do timeout -k 10 200 python bench.py --config $c --op $op --steps 10 --warmup 2 2>/dev/null | tee -a gpurun_out/r03l_ops.log | grep -o '"op": "[a-z]*"\|"value": [0-9.]*\|"frac": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' '; echo " $c"; done; done
