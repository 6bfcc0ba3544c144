#!/bin/bash
# Round 2: persistent-run kernel time vs run length, current build vs the no-tail variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02d
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 200 python scripts/runbench.py > $O/base.json 2> $O/base.err" \
 "DMT_LIB_PATH=build_variants/libdmt_earlyret.so timeout -k 10 200 python scripts/runbench.py > $O/earlyret.json 2> $O/earlyret.err"
