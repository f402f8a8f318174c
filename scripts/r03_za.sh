#!/bin/bash
# small mixed-frame batches take the 512-thread geometry: GPU suite, echo geometry, small-batch phase split
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03za}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for buf in 262144 1048576 4194304 16777216; do for o in 0 0x8000; do
  d=gpurun_out/${T}_b${buf}_o$o
  timeout -k 10 120 rocprofv3 --kernel-trace -d $PWD/$d -o run --output-format csv -- examples/echo_loopback --frames 100000 --chunk 65536 --buf $buf --opts $o > $d.log 2>&1 || { echo "FAIL $buf $o"; tail -5 $d.log; exit 1; }
  python3 - $d $buf $o <<'PY'
import csv,glob,sys,json,statistics as S
f=glob.glob(sys.argv[1]+'/**/*kernel_trace.csv',recursive=True)[0]
rows=list(csv.DictReader(open(f)))
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000 for r in rows if 'k_stream_runs' in r['Kernel_Name']]
g=[r['Grid_Size_X']+'x'+r['Workgroup_Size_X'] for r in rows if 'k_stream_runs' in r['Kernel_Name']][-1:]
j=json.loads(open(sys.argv[1]+'.log').read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[3], 'grid', g, 'calls', len(d), 'median_us', round(S.median(d),1) if d else None, 'fps', round(j['frames_per_s']), 'ok', j['ok'], 'fpb', round(j['frames_per_batch_avg']))
PY
done; done 2>&1 | tee gpurun_out/${T}_echo_geometry.txt
for sz in 262144 4194304; do for o in 0 0x8000 0x200; do
  timeout -k 10 120 python scripts/small_batch_stats.py $sz $o || exit 1
done; done 2>&1 | tee gpurun_out/${T}_small_stats.jsonl
