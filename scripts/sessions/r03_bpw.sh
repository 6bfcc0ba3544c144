#!/bin/bash
# One C2 block per workgroup (DMT_PC_BPW=1: a block's producer and consumer synchronise only with
# each other, four workgroups per CU) against four per workgroup: parity of the persistent paths,
# then the driver's command interleaved on one box.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03bpw}
mkdir -p $O
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --calls-iters 0 --repeats 10"
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
scripts/gpu_session.sh \
  "DMT_PC_BPW=1 timeout -k 10 300 $PT tests/test_gpu_parity.py -k 'mcmc_run or c2 or c1 or fetch_ll' > $O/pytest_bpw1.log 2>&1" \
  "timeout -k 10 200 $B > $O/def1.json 2> $O/def1.err" \
  "DMT_PC_BPW=1 timeout -k 10 200 $B > $O/bpw1_1.json 2> $O/bpw1_1.err" \
  "timeout -k 10 200 $B > $O/def2.json 2> $O/def2.err" \
  "DMT_PC_BPW=1 timeout -k 10 200 $B > $O/bpw1_2.json 2> $O/bpw1_2.err" \
  "timeout -k 10 200 $B > $O/def3.json 2> $O/def3.err" \
  "DMT_PC_BPW=1 timeout -k 10 200 $B > $O/bpw1_3.json 2> $O/bpw1_3.err"
