#!/bin/bash
# Round 2: canonical σ = I rule with the lane kernel's fast path: GPU suite, C5 A/B, C3 check.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02z
mkdir -p $O
NB="--no-cpu-baseline --steps 10 --warmup 3"
scripts/gpu_session.sh \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 300 python bench.py --config c5 $NB > $O/c5.json 2> $O/c5.err" \
 "DMT_LIB_PATH=build_variants/libdmt_nofast.so timeout -k 10 300 python bench.py --config c5 $NB > $O/c5_nofast.json 2> $O/c5_nofast.err" \
 "timeout -k 10 300 python bench.py --config c5 $NB > $O/c5_b.json 2> $O/c5_b.err" \
 "timeout -k 10 300 python bench.py --config c3 $NB > $O/c3.json 2> $O/c3.err"
