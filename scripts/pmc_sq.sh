#!/bin/bash
# SQ counter pass over the c3 bench (separate rocprofv3 run, --pmc only with kernel trace)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM --kernel-trace -d "$PWD/gpurun_out/pmc_sq" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc_sq.log 2>&1
echo rc=$?
