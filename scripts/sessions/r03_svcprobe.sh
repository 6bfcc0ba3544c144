#!/bin/bash
# Service latency probe: per-iteration latency of the separate-call loop, service on/off, and
# two idle windows.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03i}
mkdir -p $O
scripts/gpu_session.sh \
  "DMT_SVC_STATS=1 timeout -k 10 120 python scripts/svc_probe.py 300 > $O/probe_svc.json 2> $O/probe_svc.err" \
  "DMT_SVC_STATS=1 DMT_SVC_IDLE_MS=2 timeout -k 10 120 python scripts/svc_probe.py 300 > $O/probe_svc_idle2.json 2> $O/probe_svc_idle2.err" \
  "DMT_SERVICE=0 timeout -k 10 120 python scripts/svc_probe.py 300 > $O/probe_nosvc.json 2> $O/probe_nosvc.err"
