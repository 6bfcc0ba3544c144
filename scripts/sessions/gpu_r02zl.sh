#!/bin/bash
# Consumer loop without hoisted lane masks / Philox round keys (fewer SGPR spill reloads) vs base; parity.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zl
mkdir -p $O
A="--gpus 1 --steps 200 --warmup 20 --no-cpu-baseline"
D="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
V=build_variants/libdmt_base.so
scripts/gpu_session.sh \
 "timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k 'producer_consumer or persistent_paths or failing_blocks or mcmc_run or c2 or c1' > $O/pytest.log 2>&1" \
 "timeout -k 10 120 python bench.py $A > $O/a_new.json 2> $O/a_new.err" \
 "DMT_LIB_PATH=$V timeout -k 10 120 python bench.py $A > $O/a_base.json 2> $O/a_base.err" \
 "timeout -k 10 120 python bench.py $A > $O/a_new2.json 2> $O/a_new2.err" \
 "DMT_LIB_PATH=$V timeout -k 10 120 python bench.py $A > $O/a_base2.json 2> $O/a_base2.err" \
 "timeout -k 10 120 python bench.py $D > $O/d_new.json 2> $O/d_new.err" \
 "DMT_LIB_PATH=$V timeout -k 10 120 python bench.py $D > $O/d_base.json 2> $O/d_base.err"
