#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
B="python bench.py --config c5 --steps 3 --warmup 3 --no-cpu-baseline"
scripts/gpu_session.sh \
 "timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/f -o f --output-format csv -- $B > $O/f.log 2>&1" \
 "timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/w -o w --output-format csv -- $B > $O/w.log 2>&1" \
 "DMT_LANE_SPLIT=0 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/f0 -o f --output-format csv -- $B > $O/f0.log 2>&1" \
 "DMT_LANE_SPLIT=0 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/w0 -o w --output-format csv -- $B > $O/w0.log 2>&1"
