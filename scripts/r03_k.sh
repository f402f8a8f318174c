#!/bin/bash
# warm-up behaviour of the c3 decode: kernel time per call over 60 calls (sweep; and runs forced)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for x in 0 0x80000000; do
timeout -k 10 300 rocprofv3 --kernel-trace -d $PWD/gpurun_out/r03k_tr_$x -o run --output-format csv -- python3 bench.py --config c3 --steps 60 --warmup 1 --no-cpu --no-ceiling --xopts $x > gpurun_out/r03k_tr_$x.log 2>&1 || exit 1
python3 - $x <<'PY'
import csv,glob,sys
f=glob.glob(f'gpurun_out/r03k_tr_{sys.argv[1]}/**/*kernel_trace.csv',recursive=True)[0]
rows=sorted(csv.DictReader(open(f)), key=lambda r:int(r['Start_Timestamp']))
d=[((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000, 'S' if 'sweep' in r['Kernel_Name'] else 'R') for r in rows if 'k_stream' in r['Kernel_Name']]
print(sys.argv[1], ' '.join(f"{k}{v:.0f}" for v,k in d))
PY
done
for w in 3 30; do echo "warmup $w: $(timeout -k 10 200 python bench.py --config c3 --steps 20 --warmup $w --no-cpu --no-ceiling 2>/dev/null | grep -o '"ms_per_step": [0-9.]*')"; done
