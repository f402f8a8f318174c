# A/B of bench.py variants on one box: AB_CFGS configs x AB_ARMS ("name:xopts[:VAR=value]"), AB_REPS rounds
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-ab}
for rep in $(seq 1 ${AB_REPS:-2}); do
  for c in ${AB_CFGS:-c1 c2}; do
    for arm in ${AB_ARMS:-base:0}; do
      n=${arm%%:*}; x=${arm#*:}; ev=""
      case "$x" in *:*) ev=${x#*:}; x=${x%%:*};; esac
      timeout -k 10 200 env $ev python bench.py --config $c --no-cpu --no-ceiling --xopts $x ${AB_EXTRA:-} > gpurun_out/${T}_tmp.log 2>&1 || { echo "FAIL $c $n"; tail -5 gpurun_out/${T}_tmp.log; exit 1; }
      ms=$(tail -1 gpurun_out/${T}_tmp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("decoder",""))')
      echo "$rep $c $n $ms" | tee -a gpurun_out/${T}_ab.txt
    done
  done
done
