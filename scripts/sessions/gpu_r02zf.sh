#!/bin/bash
# Timing events created in dmt_set_timing (outside the timed region): the driver's command.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zf
mkdir -p $O
D="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
scripts/gpu_session.sh \
 "timeout -k 10 120 python bench.py $D > $O/drv1.json 2> $O/drv1.err" \
 "timeout -k 10 120 python bench.py $D > $O/drv2.json 2> $O/drv2.err" \
 "timeout -k 10 120 python bench.py $D > $O/drv3.json 2> $O/drv3.err" \
 "timeout -k 10 120 python scripts/host_overhead.py --reps 40 > $O/host.json 2> $O/host.err"
