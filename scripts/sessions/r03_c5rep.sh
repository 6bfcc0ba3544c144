#!/bin/bash
# C5 draw: tile-phase repair threshold A/B (default 1/4 vs always), same box, interleaved,
# plus the write-request count of each.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03c5rep}
mkdir -p $O
B="python bench.py --config c5 --steps 10 --warmup 3 --repeats 0 --calls-iters 0 --no-cpu-baseline"
P="TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum"
scripts/gpu_session.sh \
  "timeout -k 10 170 $B > $O/def1.json 2> $O/def1.err" \
  "DMT_REPAIR_DIV=1 timeout -k 10 170 $B > $O/rep1.json 2> $O/rep1.err" \
  "timeout -k 10 170 $B > $O/def2.json 2> $O/def2.err" \
  "DMT_REPAIR_DIV=1 timeout -k 10 170 $B > $O/rep2.json 2> $O/rep2.err" \
  "DMT_REPAIR_DIV=1 timeout -s KILL 170 rocprofv3 --pmc $P -d $O/rep_p -o p --output-format csv -- $B > $O/rep_p.log 2>&1" \
  "timeout -s KILL 170 rocprofv3 --pmc $P -d $O/def_p -o p --output-format csv -- $B > $O/def_p.log 2>&1"
