#!/bin/bash
# C2: consumer-owned trailing run steps (DMT_PC_CONS_STEPS 2, default) vs 0 and 4; parity.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zc
mkdir -p $O
A="--gpus 1 --steps 200 --warmup 20 --no-cpu-baseline"
D="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
scripts/gpu_session.sh \
 "timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k 'producer_consumer or persistent_paths or failing_blocks or mcmc_run or c2 or c1' > $O/pytest.log 2>&1" \
 "timeout -k 10 120 python bench.py $A > $O/cr2.json 2> $O/cr2.err" \
 "DMT_LIB_PATH=build_variants/libdmt_cr0.so timeout -k 10 120 python bench.py $A > $O/cr0.json 2> $O/cr0.err" \
 "DMT_LIB_PATH=build_variants/libdmt_cr4.so timeout -k 10 120 python bench.py $A > $O/cr4.json 2> $O/cr4.err" \
 "timeout -k 10 120 python bench.py $A > $O/cr2b.json 2> $O/cr2b.err" \
 "timeout -k 10 120 python bench.py $D > $O/cr2_drv.json 2> $O/cr2_drv.err" \
 "DMT_LIB_PATH=build_variants/libdmt_cr0.so timeout -k 10 120 python bench.py $D > $O/cr0_drv.json 2> $O/cr0_drv.err"
