#!/bin/bash
# Lane-kernel variants (build_variants/libdmt_<v>.so): C3 and C5 draw time, interleaved on one box.
# usage: TAG=... scripts/sessions/r03_variants.sh v1 v2 ...   ("base" = the in-tree build)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03f}
mkdir -p $O
A="--steps 30 --warmup 5 --no-cpu-baseline --repeats 0 --calls-iters 0"
steps=()
for v in "$@"; do
  lib=""
  [ "$v" != "base" ] && lib="DMT_LIB_PATH=build_variants/libdmt_$v.so"
  for c in c3 c5; do
    steps+=("$lib timeout -k 10 150 python bench.py --config $c $A > $O/${c}_$v.json 2> $O/${c}_$v.err")
  done
done
scripts/gpu_session.sh "${steps[@]}"
