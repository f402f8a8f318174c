set -e
T=${T:-r02k}
TAG=$T scripts/gpu_session.sh tests smoke pmc:c3 pmc:c2 pmc:c1 pmc:c4
for c in c3 c2 c1 c4; do python scripts/pmc_summary.py gpurun_out/${T}_pmc_${c}_fetch gpurun_out/${T}_pmc_${c}_write $c:fused ${T}_${c}_pmc; done
cp profiles/pmc_traffic.json gpurun_out/${T}_pmc_traffic.json
TAG=$T scripts/gpu_session.sh bench:c3 bench:c2 bench:c1 bench:c4 prof:c2 prof:c1 prof:c3 stats:c2
