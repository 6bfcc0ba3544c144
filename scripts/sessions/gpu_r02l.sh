#!/bin/bash
# Round 2: half-tile lane mapping (DMT_HALF_TILES) — parity under it, C3/C5 A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02l
mkdir -p $O
NB="--no-cpu-baseline --steps 10 --warmup 3"
scripts/gpu_session.sh \
 "DMT_HALF_TILES=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu_half.log 2>&1" \
 "DMT_HALF_TILES=0 timeout -k 10 300 python bench.py --config c3 $NB > $O/c3_h0.json 2> $O/c3_h0.err" \
 "DMT_HALF_TILES=1 timeout -k 10 300 python bench.py --config c3 $NB > $O/c3_h1.json 2> $O/c3_h1.err" \
 "DMT_HALF_TILES=0 timeout -k 10 300 python bench.py --config c5 $NB > $O/c5_h0.json 2> $O/c5_h0.err" \
 "DMT_HALF_TILES=1 timeout -k 10 300 python bench.py --config c5 $NB > $O/c5_h1.json 2> $O/c5_h1.err" \
 "DMT_HALF_TILES=1 DMT_LANE_SPLIT=0 timeout -k 10 300 python bench.py --config c5 $NB > $O/c5_h1_ls0.json 2> $O/c5_h1_ls0.err"
