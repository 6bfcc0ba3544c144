#!/bin/bash
# Tutorial check (docs/src/tutorials/biblock/inference.md): full GPU parity suite, a rocprofv3
# kernel trace of 300 tutorial iterations, the 10^4-iteration device chain.
# usage: scripts/gpu_tutorial.sh <outdir-name> [steps]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
N=${2:-10000}
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_tut -o tut --output-format csv -- python examples/fhn_gamma_inference.py --steps 300 --burn-in 100 > $O/prof_tut.log 2>&1" \
 "timeout -k 10 600 python -u examples/fhn_gamma_inference.py --steps $N --out $O/tutorial_device.json > $O/tutorial_device.log 2>&1" \
 "timeout -k 10 900 python -u examples/fhn_gamma_inference.py --blocking --steps $N --out $O/tutorial_blocking_device.json > $O/tutorial_blocking_device.log 2>&1"
