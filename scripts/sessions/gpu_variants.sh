#!/bin/bash
# Kernel-variant A/B on C2: bench.py (200 timed iterations) with the default build and each
# build_variants/libdmt_<v>.so named on the command line.  usage: scripts/gpu_variants.sh TAG v1 v2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
A="--gpus 1 --steps 200 --warmup 20 --no-cpu-baseline ${BENCH_ARGS}"
steps=("timeout -k 10 120 python bench.py $A > $O/base.json 2> $O/base.err")
for v in "$@"; do
  steps+=("DMT_LIB_PATH=build_variants/libdmt_$v.so timeout -k 10 120 python bench.py $A > $O/$v.json 2> $O/$v.err")
done
scripts/gpu_session.sh "${steps[@]}"
