#!/bin/bash
# Lane-kernel prefetch distance on the current kernels: K = 4 (build) vs 8 vs 16 steps per chunk
# (build_variants/libdmt_k{8,16}.so, -DDMT_KCHUNK), C3 and C5 draws with accept, interleaved on one
# box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zx
mkdir -p $O
V8="DMT_LIB_PATH=$PWD/build_variants/libdmt_k8.so"
V16="DMT_LIB_PATH=$PWD/build_variants/libdmt_k16.so"
steps=()
for r in a b; do
  for c in c5 c3; do
    K="python scripts/kbench.py --config $c --mapping lane --iters 20 --accept"
    steps+=("timeout -k 10 180 $K > $O/${c}_k4_$r.json 2> $O/${c}_k4_$r.err")
    steps+=("$V8 timeout -k 10 180 $K > $O/${c}_k8_$r.json 2> $O/${c}_k8_$r.err")
    steps+=("$V16 timeout -k 10 180 $K > $O/${c}_k16_$r.json 2> $O/${c}_k16_$r.err")
  done
done
scripts/gpu_session.sh "${steps[@]}"
