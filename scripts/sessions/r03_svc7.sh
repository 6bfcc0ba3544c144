#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03w}
mkdir -p $O
scripts/gpu_session.sh \
  "timeout -k 10 240 python -u -m pytest tests/test_deferred.py tests/test_reference_tutorials.py -m gpu -x -v --timeout 90 --timeout-method thread > $O/pytest_svc.log 2>&1" \
  "DMT_SVC_STATS=1 timeout -k 10 120 python scripts/svc_probe.py 300 > $O/probe_svc.json 2> $O/probe_svc.err" \
  "timeout -k 10 180 python bench.py --api calls --steps 500 --warmup 20 --no-cpu-baseline --repeats 0 > $O/bench_c2_calls.json 2> $O/bench_c2_calls.err"
