#!/bin/bash
# One GPU-box session: each GPU step under its own time limit; stop at the first
# step that crashed, aborted or timed out (exit codes other than 0/1).
# usage: [TAG=r02a] scripts/gpu_session.sh STEP... where STEP is one of
#   tests smoke bench bench:<cfg> stats:<cfg> prof:<cfg> pmc:<cfg> sq:<cfg> host
# Outputs land in gpurun_out/<TAG>_<step>_<cfg>.*
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
OUT=gpurun_out
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  kind=${step%%:*}; cfg=${step#*:}; [ "$cfg" = "$step" ] && cfg=c3
  n="${TAG}_${kind}_${cfg}"
  case $kind in
    tests) run "${TAG}_pytest_gpu" 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    smoke) run "${TAG}_smoke" 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run "$n" 400 python bench.py --config "$cfg" ;;
    benchq) run "$n" 300 python bench.py --config "$cfg" --no-cpu ;;
    stats) run "$n" 300 python bench.py --config "$cfg" --steps 10 --warmup 2 --no-cpu --stats ;;
    host) run "$n" 400 python bench.py --config "$cfg" --no-cpu --host-path --steps 5 ;;
    prof) run "$n" 400 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/$n" -o run --output-format csv -- python3 bench.py --config "$cfg" --steps 10 --warmup 2 --no-cpu ;;
    pmc) run "${n}_fetch" 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$PWD/$OUT/${n}_fetch" -o run --output-format csv -- python3 bench.py --config "$cfg" --steps 3 --warmup 1 --no-cpu
         run "${n}_write" 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$PWD/$OUT/${n}_write" -o run --output-format csv -- python3 bench.py --config "$cfg" --steps 3 --warmup 1 --no-cpu ;;
    sq) run "$n" 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-trace -d "$PWD/$OUT/$n" -o run --output-format csv -- python3 bench.py --config "$cfg" --steps 2 --warmup 1 --no-cpu ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
