#!/bin/bash
# Round 6: the k_utf8 probe pass (frames/echo tests + reassemble c1-c4), and
# the bound on what removing the hand-over check launch could give c1/c2
# (XYWS_OPT_LATX_ONLY = 0x80: the lattice kernel alone, timing only).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r06t}
timeout -k 10 600 python -u -m pytest tests/test_frames.py tests/test_echo_loopback.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
tail -2 gpurun_out/${T}_tests.log
summ() {
  tail -1 "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['ms_per_step'], d['roofline']['frac'], d.get('parity'))"
}
for c in c1 c2 c3 c4; do
  timeout -k 10 200 python bench.py --config $c --op reassemble --no-cpu --no-ceiling > gpurun_out/${T}_re_$c.log 2>&1
  summ gpurun_out/${T}_re_$c.log "re $c"
done
for rep in 1 2; do
  for c in c1 c2; do
    timeout -k 10 200 python bench.py --config $c --no-cpu --no-ceiling > gpurun_out/${T}_d_$c.log 2>&1
    summ gpurun_out/${T}_d_$c.log "dec $c"
    timeout -k 10 200 python bench.py --config $c --no-cpu --no-ceiling --xopts 0x80 > gpurun_out/${T}_x_$c.log 2>&1
    summ gpurun_out/${T}_x_$c.log "latonly $c"
  done
done
