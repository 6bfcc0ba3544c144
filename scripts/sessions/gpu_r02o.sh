#!/bin/bash
# Round 2: producer/consumer kernel variants (draw interleave groups, one-role stubs), C2.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02o
mkdir -p $O
A="--gpus 1 --steps 200 --warmup 20 --no-cpu-baseline"
steps=("timeout -k 10 120 python bench.py $A > $O/g1.json 2> $O/g1.err"
       "DMT_MCMC_PC=0 timeout -k 10 120 python bench.py $A > $O/w1.json 2> $O/w1.err")
for v in g2 g4 g8 stubp stubc; do
  steps+=("DMT_LIB_PATH=build_variants/libdmt_$v.so timeout -k 10 120 python bench.py $A > $O/$v.json 2> $O/$v.err")
done
scripts/gpu_session.sh "${steps[@]}"
