# A/B of bench.py between this tree and a second one (AB_OTHER, default
# ab_old: a git worktree of an earlier commit, built in place) plus option
# arms, on one box: AB_CFGS configs x arms, AB_REPS rounds. Arms:
# "name:dir:xopts" (dir "." or the other tree).
set -u
mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-abt}
ROOT=$PWD
for rep in $(seq 1 ${AB_REPS:-3}); do
  for c in ${AB_CFGS:-c1 c2}; do
    for arm in ${AB_ARMS:-new:.:0 old:ab_old:0}; do
      n=${arm%%:*}; r=${arm#*:}; d=${r%%:*}; x=${r#*:}
      (cd $ROOT/$d && timeout -k 10 200 python bench.py --config $c --no-cpu --no-ceiling --xopts $x ${AB_EXTRA:-}) > gpurun_out/${T}_tmp.log 2>&1 || { echo "FAIL $c $n"; tail -5 gpurun_out/${T}_tmp.log; exit 1; }
      ms=$(tail -1 gpurun_out/${T}_tmp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')
      echo "$rep $c $n $ms" | tee -a gpurun_out/${T}_ab.txt
    done
  done
done
