#!/bin/bash
# Round 2: cost of the persistent kernels' fetch_ll tail by phase (measurement variants).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02f
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 200 python scripts/runbench.py > $O/base.json 2> $O/base.err" \
 "DMT_LIB_PATH=build_variants/libdmt_earlyret.so timeout -k 10 200 python scripts/runbench.py > $O/earlyret.json 2> $O/earlyret.err" \
 "DMT_LIB_PATH=build_variants/libdmt_tail1.so timeout -k 10 200 python scripts/runbench.py > $O/tail1.json 2> $O/tail1.err" \
 "DMT_LIB_PATH=build_variants/libdmt_tail2.so timeout -k 10 200 python scripts/runbench.py > $O/tail2.json 2> $O/tail2.err" \
 "timeout -k 10 200 python scripts/runbench.py > $O/base2.json 2> $O/base2.err"
