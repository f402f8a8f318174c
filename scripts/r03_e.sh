#!/bin/bash
# (1) the concurrent-decode failure: HEAD library vs the working one, 3 tries each (wrong bytes, not a fault)
# (2) c3 A/B: sweep with the validation in phase B (pol) vs during the stores (v1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for lib in head v1; do for i in 1 2 3; do
  XYWS_LIB=$PWD/abl/libxyws_$lib.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "concurrent_decodes" > gpurun_out/r03e_conc_${lib}_$i.log 2>&1; echo "$lib $i rc=$? $(tail -1 gpurun_out/r03e_conc_${lib}_$i.log)"
done; done
REPS=3 CFG=c3 timeout -k 10 600 scripts/abn.sh pol=$PWD/abl/libxyws_pol.so v1=$PWD/abl/libxyws_v1.so | tee gpurun_out/r03e_ab.log
