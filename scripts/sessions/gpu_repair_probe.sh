#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r01p
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 --warmup 3 > $O/c5_d4.json 2> $O/c5_d4.err" \
 "DMT_REPAIR_DIV=2 timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 --warmup 3 > $O/c5_d2.json 2> $O/c5_d2.err" \
 "DMT_REPAIR_DIV=2 DMT_LANE_SPLIT=0 timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 --warmup 3 > $O/c5_d2_nosplit.json 2> $O/c5_d2_nosplit.err" \
 "DMT_REPAIR_DIV=2 timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 3 > $O/c3_d2.json 2> $O/c3_d2.err"
