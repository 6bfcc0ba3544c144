#!/bin/bash
# Round 4: C2 resident kernel path stores nontemporal (default) vs write-back
# (build_variants/libdmt_nont.so): C2 parity tests, the driver-command bench interleaved (the
# line's own HIP-event timed region and its event-free repeats).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04n}
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread"
BC="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --repeats 20 --calls-iters 0"
NV=build_variants/libdmt_nont.so
timeout -k 10 400 $PT tests/test_dropin.py tests/test_gpu_parity.py tests/test_deferred.py -k 'c2 or headline or mcmc_run or resident or producer or service' > $O/pytest_c2.log 2>&1 &&
timeout -k 10 150 $BC > $O/c2_nt1.json 2> $O/c2_nt1.err &&
DMT_LIB_PATH=$NV timeout -k 10 150 $BC > $O/c2_wb1.json 2> $O/c2_wb1.err &&
timeout -k 10 150 $BC > $O/c2_nt2.json 2> $O/c2_nt2.err &&
DMT_LIB_PATH=$NV timeout -k 10 150 $BC > $O/c2_wb2.json 2> $O/c2_wb2.err &&
timeout -k 10 150 $BC > $O/c2_nt3.json 2> $O/c2_nt3.err &&
DMT_LIB_PATH=$NV timeout -k 10 150 $BC > $O/c2_wb3.json 2> $O/c2_wb3.err
rc=$?
echo "session rc=$rc"
exit $rc
