cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep.py -x -v --timeout 120 --timeout-method thread -k "config_batches and (c3 or t_mixed)" > gpurun_out/r03d_sweep1.log 2>&1; rc=$?; tail -30 gpurun_out/r03d_sweep1.log; exit $rc
