#!/bin/bash
# Round 4: host-side time of the driver's C2 call with the line's timing off / stream events /
# dispatch events (scripts/host_timing.py), and the C-side split of one call (DMT_HOST_PROFILE);
# first the C2 parity tests (uniform cross-lane reads of the consumer through v_readlane).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04o}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_dropin.py tests/test_gpu_parity.py tests/test_deferred.py -k 'c2 or headline or mcmc_run or resident or producer or service' > $O/pytest_c2.log 2>&1 &&
timeout -k 10 120 python scripts/host_timing.py > $O/host_stream.json 2> $O/host_stream.err &&
DMT_DISPATCH_EVENTS=1 timeout -k 10 120 python scripts/host_timing.py > $O/host_dispatch.json 2> $O/host_dispatch.err &&
timeout -k 10 120 python scripts/host_timing.py > $O/host_stream2.json 2> $O/host_stream2.err &&
DMT_HOST_PROFILE=1 timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --repeats 5 --calls-iters 0 > $O/bench_hostprof.json 2> $O/bench_hostprof.err
rc=$?
echo "session rc=$rc"
exit $rc
