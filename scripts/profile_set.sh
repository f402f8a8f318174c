#!/bin/bash
# The profile set behind DESIGN.md §7, on the committed sources, on the GPU box:
#   TAG=r04a STEPS="tests smoke bench prof pmc ops compat host echo small" scripts/profile_set.sh
# Every step runs under its own time limit and the set stops at the first
# failing step (a GPU fault, a timeout, a failed test); outputs go to
# gpurun_out/${TAG}_*; copy the summaries worth keeping into profiles/.
#   tests   pytest -m gpu
#   smoke   __graft_entry__.smoke()
#   bench   bench.py lines for CFGS (default c3 c2 c1 c4; c3 with the CPU baseline and copy ceiling)
#   prof    rocprofv3 --kernel-trace --stats per config + steady-state summary (trace_summary.py)
#   pmc     FETCH_SIZE and WRITE_SIZE passes per config (separate runs; pmc_summary.py folds them)
#   ops     the §8(f) callers on c1-c4 (encode, classify, reassemble)
#   compat  per-header latency of the compatibility path (tests/cpp/test_compat --latency)
#   host    PCIe-inclusive host paths on c3
#   echo    the loopback echo harness at a few receive-buffer sizes
#   small   small-batch (echo-sized) decode latency with descriptors
#   valu    SQ_INSTS_VALU / SQ_WAVES of the §8(f) kernels on c2 encode and reassemble (one --pmc pass each)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r04x}
STEPS=${STEPS:-"tests bench prof pmc"}
CFGS=${CFGS:-"c3 c2 c1 c4"}
BENCH=${BENCH_ARGS:-}
step() { local n=$1 s=$2; shift 2; echo "== $n $(date +%T)"; timeout -k 10 $s "$@" > gpurun_out/${T}_$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -1 gpurun_out/${T}_$n.log | cut -c1-240; [ $rc -eq 0 ] || exit $rc; }
has() { case " $STEPS " in *" $1 "*) return 0;; esac; return 1; }
has tests && step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
has smoke && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
if has bench; then
  for c in $CFGS; do
    if [ "$c" = c3 ]; then step bench_$c 400 python bench.py --config $c $BENCH
    else step bench_$c 300 python bench.py --config $c --no-ceiling $BENCH; fi
  done
fi
if has prof; then
  for c in $CFGS; do
    step prof_$c 400 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/${T}_prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 30 --warmup 5 --no-cpu --no-ceiling $BENCH
    python scripts/trace_summary.py --skip 5 gpurun_out/${T}_prof_$c > gpurun_out/${T}_prof_${c}_summary.json
  done
fi
if has pmc; then
  for c in $CFGS; do
    step pmcf_$c 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $PWD/gpurun_out/${T}_pmc_${c}_fetch -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 3 --settle 0 --no-cpu --no-ceiling $BENCH
    step pmcw_$c 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $PWD/gpurun_out/${T}_pmc_${c}_write -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 3 --settle 0 --no-cpu --no-ceiling $BENCH
  done
fi
if has ops; then
  for c in c3 c2 c1 c4; do for op in encode classify reassemble; do
    step op_${op}_$c 300 python bench.py --config $c --op $op --no-cpu --no-ceiling
  done; done
fi
has compat && step compat 120 tests/cpp/test_compat --latency
has host && step host_c3 400 python bench.py --config c3 --no-cpu --no-ceiling --host-path --steps 5
if has echo; then
  for b in 262144 4194304; do step echo_$b 200 examples/echo_loopback --frames 200000 --buf $b; done
fi
has small && step small 300 python scripts/small_batch_stats.py
if has valu; then
  for op in encode reassemble; do
    step valu_$op 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --kernel-trace -d $PWD/gpurun_out/${T}_valu_$op -o run --output-format csv -- python3 bench.py --config c2 --op $op --steps 3 --warmup 2 --no-cpu --no-ceiling
  done
fi
echo "== done $T"
