#!/bin/bash
# One GPU-box session: each GPU step under its own time limit; stop at the first
# step that crashed, aborted or timed out (exit codes other than 0/1).
# usage: scripts/gpu_session.sh STEP... where STEP is one of
#   tests smoke bench bench_c2 bench_c4 prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    tests_all) run pytest_gpu 1200 python -m pytest tests -m gpu -q ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    bench_quick) run bench_quick 300 python bench.py --steps 10 --warmup 2 --no-cpu --stats ;;
    bench_c2) run bench_c2 300 python bench.py --config c2 --no-cpu ;;
    bench_c1) run bench_c1 300 python bench.py --config c1 --no-cpu ;;
    bench_c4) run bench_c4 300 python bench.py --config c4 --no-cpu ;;
    host) run bench_host 600 python bench.py --no-cpu --host-path --steps 5 ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu ;;
    pmc_fetch) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$PWD/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu ;;
    pmc_write) run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$PWD/gpurun_out/pmc_write" -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
