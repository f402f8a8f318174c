#!/bin/bash
# A/B timing of decoder library builds from git revisions (diagnostic, not product).
#   here:    scripts/ab.sh build REV...      (builds exp/libxyws_<rev>.so from that revision's sources)
#   GPU box: scripts/ab.sh run REV...        (CFGS="c3 c2", REPS=2: bench each build in turn)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mode=$1; shift
if [ "$mode" = variant ]; then  # scripts/ab.sh variant NAME "-DFLAG=..." : the working tree's sources
  name=$1; shift
  mkdir -p exp
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-function \
    -Iinclude -Ixynet_amd/csrc $@ xynet_amd/csrc/xyws.hip xynet_amd/csrc/xyws_stream.hip xynet_amd/csrc/xyws_frames.hip \
    xynet_amd/csrc/xyws_arena.hip -o "exp/libxyws_$name.so" || exit 1
  echo "built exp/libxyws_$name.so"; exit 0
fi
if [ "$mode" = build ]; then
  mkdir -p exp
  for rev in "$@"; do
    d=exp/src_$rev; rm -rf "$d"; mkdir -p "$d/include" "$d/csrc"
    git show "$rev:include/xyws.h" > "$d/include/xyws.h" || exit 1
    git show "$rev:include/xyws_synth.h" > "$d/include/xyws_synth.h" 2>/dev/null
    srcs=""
    for f in $(git ls-tree --name-only "$rev" xynet_amd/csrc/); do
      f=$(basename "$f"); git show "$rev:xynet_amd/csrc/$f" > "$d/csrc/$f" || exit 1
      case $f in *.hip) [ "$f" != xyws_tools.hip ] && srcs="$srcs $d/csrc/$f";; esac
    done
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-function \
      -I"$d/include" -I"$d/csrc" $srcs -o "exp/libxyws_$rev.so" || exit 1
    echo "built exp/libxyws_$rev.so"
  done
  exit 0
fi
for rep in $(seq ${REPS:-2}); do
  for rev in "$@"; do
    for cfg in ${CFGS:-c3}; do
      lib=$PWD/exp/libxyws_$rev.so; [ "$rev" = cur ] && lib=$PWD/xynet_amd/libxyws.so
      echo "$rev $cfg $(XYWS_LIB=$lib timeout -k 10 120 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu 2>/dev/null | grep -o '"ms_per_step": [0-9.]*\|"kernel_ms_avg": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' ')"
    done
  done
done
