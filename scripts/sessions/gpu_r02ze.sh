#!/bin/bash
# Completion marker after a timed run (DMT_DONE_EVENT) and consumer-drawn run steps 1/3 vs 2.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02ze
mkdir -p $O
A="--gpus 1 --steps 200 --warmup 20 --no-cpu-baseline"
D="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
scripts/gpu_session.sh \
 "timeout -k 10 120 python scripts/host_overhead.py --reps 40 > $O/host_d0.json 2> $O/host_d0.err" \
 "DMT_DONE_EVENT=1 timeout -k 10 120 python scripts/host_overhead.py --reps 40 > $O/host_d1.json 2> $O/host_d1.err" \
 "DMT_DONE_EVENT=2 timeout -k 10 120 python scripts/host_overhead.py --reps 40 > $O/host_d2.json 2> $O/host_d2.err" \
 "DMT_DISPATCH_EVENTS=0 timeout -k 10 120 python scripts/host_overhead.py --reps 40 > $O/host_r0.json 2> $O/host_r0.err" \
 "DMT_DISPATCH_EVENTS=0 DMT_DONE_EVENT=2 timeout -k 10 120 python scripts/host_overhead.py --reps 40 > $O/host_r2.json 2> $O/host_r2.err" \
 "timeout -k 10 120 python bench.py $D > $O/drv_d0.json 2> $O/drv_d0.err" \
 "DMT_DONE_EVENT=1 timeout -k 10 120 python bench.py $D > $O/drv_d1.json 2> $O/drv_d1.err" \
 "DMT_DONE_EVENT=2 timeout -k 10 120 python bench.py $D > $O/drv_d2.json 2> $O/drv_d2.err" \
 "timeout -k 10 120 python bench.py $A > $O/cr2.json 2> $O/cr2.err" \
 "DMT_LIB_PATH=build_variants/libdmt_cr1.so timeout -k 10 120 python bench.py $A > $O/cr1.json 2> $O/cr1.err" \
 "DMT_LIB_PATH=build_variants/libdmt_cr3.so timeout -k 10 120 python bench.py $A > $O/cr3.json 2> $O/cr3.err" \
 "timeout -k 10 120 python bench.py $A > $O/cr2b.json 2> $O/cr2b.err"
