#!/bin/bash
# Service latency: in-tree build vs the same source built in one hipcc call (plain) vs the
# stage-probe build, interleaved.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03t}
mkdir -p $O
steps=()
for k in 1 2; do
  steps+=("timeout -k 10 120 python scripts/svc_probe.py 300 > $O/intree_$k.json 2> $O/intree_$k.err")
  steps+=("DMT_LIB_PATH=build_variants/plain/libdmt.so timeout -k 10 120 python scripts/svc_probe.py 300 > $O/plain_$k.json 2> $O/plain_$k.err")
  steps+=("DMT_LIB_PATH=build_variants/svcprobe/libdmt.so timeout -k 10 120 python scripts/svc_probe.py 300 > $O/probe_$k.json 2> $O/probe_$k.err")
done
scripts/gpu_session.sh "${steps[@]}"
