#!/bin/bash
# A/B timing of compile-time variants of libxyws.so (diagnostic, not product):
# build here with  scripts/exp_variants.sh build "NAME:-DFLAGS ..." ...
# run on the box:  scripts/exp_variants.sh run NAME... (CFGS="c3 c1")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mode=$1; shift
if [ "$mode" = build ]; then
  for v in "$@"; do
    name=${v%%:*}; flags=${v#*:}
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -falign-loops=64 -std=c++17 -fPIC -shared -Wno-unused-function \
      -Iinclude -Ixynet_amd/csrc $flags xynet_amd/csrc/xyws.hip xynet_amd/csrc/xyws_stream.hip \
      xynet_amd/csrc/xyws_frames.hip xynet_amd/csrc/xyws_arena.hip -o exp/libxyws_$name.so || exit 1
  done
  exit 0
fi
for rep in $(seq ${REPS:-2}); do
for name in "$@"; do
  for cfg in ${CFGS:-c3 c1}; do
    lib=$PWD/exp/libxyws_$name.so; [ "$name" = cur ] && lib=$PWD/xynet_amd/libxyws.so
    echo "$name $cfg $(XYWS_LIB=$lib timeout -k 10 120 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' ')"
  done
done
done
