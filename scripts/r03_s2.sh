#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 scripts/bw_probe6 > gpurun_out/r03b_probe6.log 2>&1; rc=$?; cat gpurun_out/r03b_probe6.log; [ $rc -eq 0 ] || exit $rc
REPS=4 timeout -k 10 400 scripts/abn.sh base=$PWD/abl/libxyws_base.so fence=cur | tee gpurun_out/r03b_ab_fence.log
