#!/bin/bash
# Round 2: two-level arrival trees for the persistent runs' fetch_ll.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02i
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 200 python scripts/runbench.py > $O/base.json 2> $O/base.err" \
 "DMT_LIB_PATH=build_variants/libdmt_earlyret.so timeout -k 10 200 python scripts/runbench.py > $O/earlyret.json 2> $O/earlyret.err" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2_driver.json 2> $O/bench_c2_driver.err"
