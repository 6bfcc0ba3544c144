#!/bin/bash
# Service: parity tests, latency probe (in-tree build), stage probe (svcprobe variant).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03m}
mkdir -p $O
scripts/gpu_session.sh \
  "timeout -k 10 240 python -u -m pytest tests/test_deferred.py -m gpu -x -v --timeout 90 --timeout-method thread > $O/pytest_svc.log 2>&1" \
  "DMT_SVC_STATS=1 timeout -k 10 120 python scripts/svc_probe.py 300 > $O/probe_svc.json 2> $O/probe_svc.err" \
  "DMT_LIB_PATH=build_variants/svcprobe/libdmt.so timeout -k 10 120 python scripts/svc_probe.py 300 > $O/probe_stages.json 2> $O/probe_stages.err"
