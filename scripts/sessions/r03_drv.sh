#!/bin/bash
# The driver's command three times (first-call effects), then the service probe.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03drv}
mkdir -p $O
scripts/gpu_session.sh \
  "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv1.json 2> $O/drv1.err" \
  "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv2.json 2> $O/drv2.err" \
  "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv3.json 2> $O/drv3.err"
