#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03n}
mkdir -p $O
scripts/gpu_session.sh \
  "DMT_LIB_PATH=build_variants/svcprobe/libdmt.so timeout -k 10 120 python scripts/svc_probe.py 300 > $O/probe_stages.json 2> $O/probe_stages.err"
