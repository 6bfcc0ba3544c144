#!/bin/bash
# Round 2: fp32 normal stream with 4 normals per Philox block: GPU suite, C5/C3 benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02m
mkdir -p $O
NB="--no-cpu-baseline --steps 10 --warmup 3"
scripts/gpu_session.sh \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 300 python bench.py --config c5 $NB > $O/c5.json 2> $O/c5.err" \
 "DMT_LANE_SPLIT=0 timeout -k 10 300 python bench.py --config c5 $NB > $O/c5_ls0.json 2> $O/c5_ls0.err" \
 "timeout -k 10 300 python bench.py --config c3 $NB > $O/c3.json 2> $O/c3.err"
