#!/bin/bash
# Round 4: OU time-dependent dmt_mcmc_run on the per-iteration kernels (isolated first, launches
# synchronous so that a fault names its call); C2 producer/consumer set-up with the first
# normals drawn while the set-up loads are in flight (default) vs after them
# (build_variants/libdmt_noovl.so): driver-command bench interleaved, device stamps of both;
# the time-dependent tests and the GPU suite.  Stops at the first failing step.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04i}
mkdir -p $O
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread"
BC="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --repeats 20 --calls-iters 0"
NV=build_variants/libdmt_noovl.so
HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 $PT tests/test_td_aux.py -k ou_td_aux_mcmc_run > $O/pytest_ou_mcmc.log 2>&1 &&
DMT_LIB_PATH=build_variants/libdmt_stamps.so timeout -k 10 120 python scripts/pc_stamps.py > $O/c2_stamps.jsonl 2> $O/c2_stamps.err &&
DMT_LIB_PATH=build_variants/libdmt_stamps0.so timeout -k 10 120 python scripts/pc_stamps.py > $O/c2_stamps0.jsonl 2> $O/c2_stamps0.err &&
timeout -k 10 150 $BC > $O/c2_ovl1.json 2> $O/c2_ovl1.err &&
DMT_LIB_PATH=$NV timeout -k 10 150 $BC > $O/c2_noovl1.json 2> $O/c2_noovl1.err &&
timeout -k 10 150 $BC > $O/c2_ovl2.json 2> $O/c2_ovl2.err &&
DMT_LIB_PATH=$NV timeout -k 10 150 $BC > $O/c2_noovl2.json 2> $O/c2_noovl2.err &&
timeout -k 10 300 $PT tests/test_td_aux.py > $O/pytest_td.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "session rc=$rc"
exit $rc
