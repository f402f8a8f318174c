#!/bin/bash
# dense0 hint (run decoder: dense pass from each run's first segment after a call of small mixed-size
# frames): full GPU suite, echo batches at several buffer sizes with / without it (and WG512), c1-c4 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03z}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for buf in 262144 1048576 4194304 16777216; do for o in 0 0x1000 0x40000; do
  d=gpurun_out/${T}_b${buf}_o$o
  timeout -k 10 120 rocprofv3 --kernel-trace -d $PWD/$d -o run --output-format csv -- examples/echo_loopback --frames 100000 --chunk 65536 --buf $buf --opts $o > $d.log 2>&1 || { echo "FAIL $buf $o"; tail -5 $d.log; exit 1; }
  python3 - $d $buf $o <<'PY'
import csv,glob,sys,json,statistics as S
f=glob.glob(sys.argv[1]+'/**/*kernel_trace.csv',recursive=True)[0]
rows=list(csv.DictReader(open(f)))
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000 for r in rows if 'k_stream_runs' in r['Kernel_Name']]
g=[r['Grid_Size_X'] for r in rows if 'k_stream_runs' in r['Kernel_Name']][:1]
j=json.loads(open(sys.argv[1]+'.log').read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[3], 'grid', g, 'calls', len(d), 'median_us', round(S.median(d),1) if d else None, 'fps', round(j['frames_per_s']), 'ok', j['ok'], 'fpb', round(j['frames_per_batch_avg']))
PY
done; done 2>&1 | tee gpurun_out/${T}_echo_geometry.txt
for c in c4 c2 c1; do for i in 1 2; do for x in 0 0x1000; do
  r=$(timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --no-cpu --no-ceiling --xopts $x 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' ')
  [ -n "$r" ] || { echo "bench $c $x FAILED"; exit 3; }
  echo "$c $x $i $r"
done; done; done 2>&1 | tee gpurun_out/${T}_ab.txt
