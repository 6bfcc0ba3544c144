#!/bin/bash
# C3 probe: the chunk's X°/W° rows as 16-byte stores (build_variants/libdmt_widest.so, timing
# only: the rows land permuted) against the default per-row 4-byte stores, same box, interleaved.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03widec3}
mkdir -p $O
B="python bench.py --config c3 --steps 10 --warmup 3 --repeats 0 --calls-iters 0 --no-cpu-baseline"
V=DMT_LIB_PATH=build_variants/libdmt_widest.so
P="TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum"
scripts/gpu_session.sh \
  "timeout -k 10 170 $B > $O/def1.json 2> $O/def1.err" \
  "$V timeout -k 10 170 $B > $O/wide1.json 2> $O/wide1.err" \
  "timeout -k 10 170 $B > $O/def2.json 2> $O/def2.err" \
  "$V timeout -k 10 170 $B > $O/wide2.json 2> $O/wide2.err" \
  "$V timeout -s KILL 170 rocprofv3 --pmc $P -d $O/wide_p -o p --output-format csv -- $B > $O/wide_p.log 2>&1"
