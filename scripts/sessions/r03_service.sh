#!/bin/bash
# Resident service: its parity tests first (short limits), then the deferred tests with the
# service off, then the separate-call loop with the service on / off.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03h}
mkdir -p $O
scripts/gpu_session.sh \
  "timeout -k 10 240 python -u -m pytest tests/test_deferred.py -m gpu -x -v --timeout 90 --timeout-method thread > $O/pytest_svc.log 2>&1" \
  "DMT_SERVICE=0 timeout -k 10 240 python -u -m pytest tests/test_deferred.py -m gpu -x -v --timeout 90 --timeout-method thread > $O/pytest_nosvc.log 2>&1" \
  "timeout -k 10 180 python bench.py --api calls --steps 500 --warmup 20 --no-cpu-baseline --repeats 0 > $O/bench_c2_calls.json 2> $O/bench_c2_calls.err" \
  "DMT_SERVICE=0 timeout -k 10 180 python bench.py --api calls --steps 500 --warmup 20 --no-cpu-baseline --repeats 0 > $O/bench_c2_calls_nosvc.json 2> $O/bench_c2_calls_nosvc.err"
