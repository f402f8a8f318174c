#!/bin/bash
# Copy one profile session's results (TAG) from gpurun_out/ into profiles/ and stamp the PMC traffic
# (run here, after the GPU call, on the same sources the call profiled)
set -eu
cd "$(dirname "$0")/.."
T=${1:?tag}
for c in c3 c2 c1 c4; do
  python scripts/pmc_summary.py gpurun_out/${T}_pmc_${c}_fetch gpurun_out/${T}_pmc_${c}_write $c:fused ${T}_${c}_pmc > /dev/null
  grep '^{' gpurun_out/${T}_bench_$c.log | tail -1 > profiles/${T}_${c}_bench.json
  cp gpurun_out/${T}_prof_$c/run_kernel_stats.csv profiles/${T}_${c}_kernel_stats.csv
  cp gpurun_out/${T}_prof_${c}_summary.json profiles/${T}_${c}_kernel_steady.json
  cp gpurun_out/${T}_pmc_${c}_fetch/run_counter_collection.csv profiles/${T}_${c}_pmc_fetch.csv
  cp gpurun_out/${T}_pmc_${c}_write/run_counter_collection.csv profiles/${T}_${c}_pmc_write.csv
done
grep '^{' gpurun_out/${T}_host_c3.log | tail -1 > profiles/${T}_c3_host_path.json
cp gpurun_out/${T}_compat.log profiles/${T}_compat_latency.txt
for f in gpurun_out/${T}_op_*.log; do [ -e "$f" ] && grep '^{' "$f" | tail -1; done > profiles/${T}_ops.jsonl || true
[ -d gpurun_out/${T}_prof_ops_c3 ] && cp gpurun_out/${T}_prof_ops_c3/run_kernel_stats.csv profiles/${T}_encode_c3_kernel_stats.csv
for f in gpurun_out/${T}_echo_*.log; do [ -e "$f" ] && grep '^{' "$f" | tail -1; done > profiles/${T}_echo_loopback.jsonl || true
[ -d gpurun_out/${T}_echo_prof ] && cp gpurun_out/${T}_echo_prof/run_kernel_stats.csv profiles/${T}_echo_kernel_stats.csv
[ -e gpurun_out/${T}_small_stats.jsonl ] && cp gpurun_out/${T}_small_stats.jsonl profiles/${T}_small_batch_stats.jsonl
cp gpurun_out/${T}_tests.log profiles/${T}_gpu_tests_tail.txt && python - "$T" <<'PY'
import sys
p=f"profiles/{sys.argv[1]}_gpu_tests_tail.txt"
l=open(p).read().splitlines()
open(p,"w").write("\n".join(l[-5:])+"\n")
PY
echo collected $T
