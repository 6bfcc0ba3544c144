#!/bin/bash
# First timed call with primed vs fresh timing events; the driver's command.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zh
mkdir -p $O
D="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
scripts/gpu_session.sh \
 "timeout -k 10 120 python scripts/first_call_probe.py > $O/fc_p1.json 2> $O/fc_p1.err" \
 "DMT_EVENT_PRIME=0 timeout -k 10 120 python scripts/first_call_probe.py > $O/fc_p0.json 2> $O/fc_p0.err" \
 "timeout -k 10 120 python scripts/first_call_probe.py > $O/fc_p1b.json 2> $O/fc_p1b.err" \
 "DMT_EVENT_PRIME=0 timeout -k 10 120 python scripts/first_call_probe.py > $O/fc_p0b.json 2> $O/fc_p0b.err" \
 "timeout -k 10 120 python bench.py $D > $O/drv1.json 2> $O/drv1.err" \
 "timeout -k 10 120 python bench.py $D > $O/drv2.json 2> $O/drv2.err" \
 "DMT_EVENT_PRIME=0 timeout -k 10 120 python bench.py $D > $O/drv_p0.json 2> $O/drv_p0.err"
