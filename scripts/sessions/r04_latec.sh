#!/bin/bash
# Round 4: C2 consumer forming its own steps' next proposal after B2 (default) vs before it
# (build_variants/libdmt_latec0.so): C2 parity tests, per-iteration stamps, the
# driver-command bench interleaved.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04m}
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread"
BC="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --repeats 20 --calls-iters 0"
NV=build_variants/libdmt_latec0.so
timeout -k 10 400 $PT tests/test_dropin.py tests/test_gpu_parity.py tests/test_deferred.py -k 'c2 or headline or mcmc_run or resident or producer or service' > $O/pytest_c2.log 2>&1 &&
DMT_LIB_PATH=build_variants/libdmt_stamps.so timeout -k 10 120 python scripts/pc_stamps.py > $O/c2_stamps.jsonl 2> $O/c2_stamps.err &&
timeout -k 10 150 $BC > $O/c2_latec1.json 2> $O/c2_latec1.err &&
DMT_LIB_PATH=$NV timeout -k 10 150 $BC > $O/c2_latec0_1.json 2> $O/c2_latec0_1.err &&
timeout -k 10 150 $BC > $O/c2_latec2.json 2> $O/c2_latec2.err &&
DMT_LIB_PATH=$NV timeout -k 10 150 $BC > $O/c2_latec0_2.json 2> $O/c2_latec0_2.err &&
timeout -k 10 150 $BC > $O/c2_latec3.json 2> $O/c2_latec3.err &&
DMT_LIB_PATH=$NV timeout -k 10 150 $BC > $O/c2_latec0_3.json 2> $O/c2_latec0_3.err
rc=$?
echo "session rc=$rc"
exit $rc
