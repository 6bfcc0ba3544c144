#!/bin/bash
# The bench's timed call repeated: first call vs later ones, with and without idle gaps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zg
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 120 python scripts/first_call_probe.py > $O/fc0.json 2> $O/fc0.err" \
 "timeout -k 10 120 python scripts/first_call_probe.py --idle-ms 5 > $O/fc5.json 2> $O/fc5.err" \
 "timeout -k 10 120 python scripts/first_call_probe.py --idle-ms 50 > $O/fc50.json 2> $O/fc50.err" \
 "timeout -k 10 120 python scripts/first_call_probe.py --steps 200 --warmup 20 > $O/fc200.json 2> $O/fc200.err"
