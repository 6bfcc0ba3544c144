#!/bin/bash
# Quick GPU check: parity tests (optionally a -k filter: $2), the C2 bench, kernel trace.
# usage: scripts/gpu_quick.sh <outdir-name> [pytest -k expr]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
K=""; [ -n "$2" ] && K="-k '$2'"
scripts/gpu_session.sh \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread $K > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py --steps 50 --no-cpu-baseline > $O/prof_c2.log 2>&1"
