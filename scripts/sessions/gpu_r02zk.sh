#!/bin/bash
# C5 draw time with uniform vs mixed selectors: what the partial-sector write amplification costs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zk
mkdir -p $O
K="python scripts/kbench.py --config c5 --mapping lane --iters 20"
scripts/gpu_session.sh \
 "timeout -k 10 180 $K > $O/c5_uniform.json 2> $O/c5_uniform.err" \
 "timeout -k 10 180 $K --accept > $O/c5_mixed.json 2> $O/c5_mixed.err" \
 "timeout -k 10 180 $K --accept-all > $O/c5_allacc.json 2> $O/c5_allacc.err" \
 "DMT_REPAIR_DIV=2 timeout -k 10 180 $K --accept > $O/c5_mixed_rep2.json 2> $O/c5_mixed_rep2.err" \
 "timeout -k 10 180 $K > $O/c5_uniform_b.json 2> $O/c5_uniform_b.err" \
 "timeout -k 10 180 $K --accept > $O/c5_mixed_b.json 2> $O/c5_mixed_b.err"
