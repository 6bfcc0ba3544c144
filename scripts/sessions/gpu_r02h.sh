#!/bin/bash
# Round 2: persistent-run kernel time, current build vs the no-tail variant, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02h
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 200 python scripts/runbench.py > $O/base.json 2> $O/base.err" \
 "DMT_LIB_PATH=build_variants/libdmt_earlyret.so timeout -k 10 200 python scripts/runbench.py > $O/earlyret.json 2> $O/earlyret.err" \
 "timeout -k 10 200 python scripts/runbench.py > $O/base2.json 2> $O/base2.err" \
 "DMT_LIB_PATH=build_variants/libdmt_earlyret.so timeout -k 10 200 python scripts/runbench.py > $O/earlyret2.json 2> $O/earlyret2.err" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2_driver.json 2> $O/bench_c2_driver.err"
