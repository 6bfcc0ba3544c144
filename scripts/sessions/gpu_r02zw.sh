#!/bin/bash
# Bench lines on the final build after the C3 counter summaries landed: the driver's C2 command
# and C3 (its line now carries the hbm-latency issue summary), each with its CPU leg.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zw
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err" \
 "timeout -k 10 400 python bench.py --config c3 --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err"
