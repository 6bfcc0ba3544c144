#!/bin/bash
# Round 2: table-driven fp64 Box–Muller: full GPU suite, benches C2 (driver command + 200 it), C3, C5.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02q
mkdir -p $O
NB="--no-cpu-baseline"
scripts/gpu_session.sh \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 $NB > $O/c2.json 2> $O/c2.err" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 $NB > $O/c2_200.json 2> $O/c2_200.err" \
 "timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 $NB > $O/c3.json 2> $O/c3.err" \
 "timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 $NB > $O/c5.json 2> $O/c5.err"
