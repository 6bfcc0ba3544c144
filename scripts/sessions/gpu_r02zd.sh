#!/bin/bash
# Timing-event flags: host cost of one dmt_mcmc_run call and the driver's bench command.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zd
mkdir -p $O
D="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
scripts/gpu_session.sh \
 "timeout -k 10 120 python scripts/host_overhead.py --reps 40 > $O/host_f0.json 2> $O/host_f0.err" \
 "DMT_EVENT_FLAGS=0x20000000 timeout -k 10 120 python scripts/host_overhead.py --reps 40 > $O/host_f2.json 2> $O/host_f2.err" \
 "DMT_EVENT_FLAGS=0x60000000 timeout -k 10 120 python scripts/host_overhead.py --reps 40 > $O/host_f6.json 2> $O/host_f6.err" \
 "DMT_DISPATCH_EVENTS=0 DMT_EVENT_FLAGS=0x60000000 timeout -k 10 120 python scripts/host_overhead.py --reps 40 > $O/host_r6.json 2> $O/host_r6.err" \
 "timeout -k 10 120 python bench.py $D > $O/drv_f0.json 2> $O/drv_f0.err" \
 "DMT_EVENT_FLAGS=0x20000000 timeout -k 10 120 python bench.py $D > $O/drv_f2.json 2> $O/drv_f2.err" \
 "DMT_EVENT_FLAGS=0x60000000 timeout -k 10 120 python bench.py $D > $O/drv_f6.json 2> $O/drv_f6.err" \
 "DMT_DISPATCH_EVENTS=0 DMT_EVENT_FLAGS=0x60000000 timeout -k 10 120 python bench.py $D > $O/drv_r6.json 2> $O/drv_r6.err" \
 "timeout -k 10 120 python bench.py $D > $O/drv_f0b.json 2> $O/drv_f0b.err" \
 "DMT_EVENT_FLAGS=0x20000000 timeout -k 10 120 python bench.py $D > $O/drv_f2b.json 2> $O/drv_f2b.err"
