#!/bin/bash
# Round 2: coalesced last-arriver trees, pinned per-iteration results, spin-sync option.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02e
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 200 python scripts/runbench.py > $O/run_base.json 2> $O/run_base.err" \
 "DMT_SYNC_SPIN=1 timeout -k 10 200 python scripts/runbench.py > $O/run_spin.json 2> $O/run_spin.err" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2_driver.json 2> $O/bench_c2_driver.err" \
 "DMT_SYNC_SPIN=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2_driver_spin.json 2> $O/bench_c2_driver_spin.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2drv -o c2 --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_c2drv.log 2>&1"
