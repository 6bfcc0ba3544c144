#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r01u
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k 'c3 or c5 or ragged or device_rng' > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 --warmup 3 > $O/c5_split.json 2> $O/c5_split.err" \
 "DMT_LANE_SPLIT=1 timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 3 > $O/c3_split.json 2> $O/c3_split.err" \
 "timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 3 > $O/c3_nosplit.json 2> $O/c3_nosplit.err"
