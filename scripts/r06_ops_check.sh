#!/bin/bash
# Round 6: the §8(f) callers — frames/echo GPU tests, then bench.py --op
# encode / reassemble on c1-c4 (one JSON line each into ${T}_ops.jsonl).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r06u}
timeout -k 10 600 python -u -m pytest tests/test_frames.py tests/test_echo_loopback.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_ops.jsonl
for op in ${OPS:-encode reassemble}; do
  for c in ${CFGS:-c1 c2 c3 c4}; do
    timeout -k 10 200 python bench.py --config $c --op $op --no-cpu --no-ceiling > gpurun_out/${T}_tmp.log 2>&1
    tail -1 gpurun_out/${T}_tmp.log >> gpurun_out/${T}_ops.jsonl
    tail -1 gpurun_out/${T}_tmp.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$op $c', d['ms_per_step'], d['roofline']['frac'], d.get('parity'))"
  done
done
