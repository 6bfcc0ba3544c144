#!/bin/bash
# Recorded timing events (new default) vs dispatch-attached events: the driver's command, and the
# rocprofv3 kernel trace of the same command.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zp
mkdir -p $O
D="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
scripts/gpu_session.sh \
 "timeout -k 10 120 python bench.py $D > $O/d_rec1.json 2> $O/d_rec1.err" \
 "DMT_DISPATCH_EVENTS=1 timeout -k 10 120 python bench.py $D > $O/d_disp1.json 2> $O/d_disp1.err" \
 "timeout -k 10 120 python bench.py $D > $O/d_rec2.json 2> $O/d_rec2.err" \
 "DMT_DISPATCH_EVENTS=1 timeout -k 10 120 python bench.py $D > $O/d_disp2.json 2> $O/d_disp2.err" \
 "timeout -k 10 120 python bench.py $D > $O/d_rec3.json 2> $O/d_rec3.err" \
 "DMT_DISPATCH_EVENTS=1 timeout -k 10 120 python bench.py $D > $O/d_disp3.json 2> $O/d_disp3.err" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err" \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py $D > $O/prof_c2.log 2>&1"
