#!/bin/bash
# Lane mapping with / without the producer/consumer split (k_block_ps): GPU tests, C5 and C3 benches.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r01m
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 --warmup 3 > $O/c5_split.json 2> $O/c5_split.err" \
 "DMT_LANE_SPLIT=0 timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 --warmup 3 > $O/c5_nosplit.json 2> $O/c5_nosplit.err" \
 "DMT_LANE_SPLIT=1 timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 3 > $O/c3_split.json 2> $O/c3_split.err" \
 "timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 3 > $O/c3_nosplit.json 2> $O/c3_nosplit.err"
