#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03u}
mkdir -p $O
steps=("timeout -k 10 60 python scripts/numa_info.py > $O/numa.json 2> $O/numa.err")
for k in 1 2; do
  for pin in local remote none; do
    e=""; [ $pin != none ] && e="SVC_PIN=$pin"
    steps+=("$e timeout -k 10 120 python scripts/svc_probe.py 300 > $O/${pin}_$k.json 2> $O/${pin}_$k.err")
  done
done
scripts/gpu_session.sh "${steps[@]}"
