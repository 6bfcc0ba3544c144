#!/bin/bash
# Service stage probe (build_variants/svcprobe: DMT_SVC_PROBE stamps).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03l}
mkdir -p $O
scripts/gpu_session.sh \
  "DMT_LIB_PATH=build_variants/svcprobe/libdmt.so DMT_SVC_STATS=1 timeout -k 10 120 python scripts/svc_probe.py 300 > $O/probe_svc.json 2> $O/probe_svc.err"
