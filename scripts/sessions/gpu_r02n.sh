#!/bin/bash
# Round 2: producer/consumer split of the resident C2 kernel: parity tests, A/B bench, kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02n
mkdir -p $O
NB="--no-cpu-baseline"
scripts/gpu_session.sh \
 "timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k 'producer_consumer or persistent_paths or failing_blocks' > $O/pytest_pc.log 2>&1" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 $NB > $O/c2_pc.json 2> $O/c2_pc.err" \
 "DMT_MCMC_PC=0 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 $NB > $O/c2_1w.json 2> $O/c2_1w.err" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 500 --warmup 20 $NB > $O/c2_pc_500.json 2> $O/c2_pc_500.err" \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 $NB > $O/prof_c2.log 2>&1"
