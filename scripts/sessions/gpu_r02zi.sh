#!/bin/bash
# Write-through (sc1) X°/W° stores in the resident PC kernel vs plain (DMT_PC_WT=0); parity.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zi
mkdir -p $O
A="--gpus 1 --steps 200 --warmup 20 --no-cpu-baseline"
D="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
V=build_variants/libdmt_wt0.so
scripts/gpu_session.sh \
 "timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k 'producer_consumer or persistent_paths or failing_blocks or mcmc_run or c2 or c1' > $O/pytest.log 2>&1" \
 "timeout -k 10 120 python bench.py $D > $O/drv_wt1.json 2> $O/drv_wt1.err" \
 "DMT_LIB_PATH=$V timeout -k 10 120 python bench.py $D > $O/drv_wt0.json 2> $O/drv_wt0.err" \
 "timeout -k 10 120 python bench.py $D > $O/drv_wt1b.json 2> $O/drv_wt1b.err" \
 "DMT_LIB_PATH=$V timeout -k 10 120 python bench.py $D > $O/drv_wt0b.json 2> $O/drv_wt0b.err" \
 "timeout -k 10 120 python bench.py $A > $O/a_wt1.json 2> $O/a_wt1.err" \
 "DMT_LIB_PATH=$V timeout -k 10 120 python bench.py $A > $O/a_wt0.json 2> $O/a_wt0.err" \
 "timeout -k 10 120 python scripts/first_call_probe.py > $O/fc_wt1.json 2> $O/fc_wt1.err" \
 "DMT_LIB_PATH=$V timeout -k 10 120 python scripts/first_call_probe.py > $O/fc_wt0.json 2> $O/fc_wt0.err"
