#!/bin/bash
# A/B timing of decoder variants (diagnostic; one GPU session)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in ${CFGS:-c3 c2 c4}; do
  for x in ${XOPTS:-0 0x40000}; do
    echo "$cfg xopts=$x $(timeout -k 10 120 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu --xopts $x 2>/dev/null | grep -o '"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' ')"
  done
done
