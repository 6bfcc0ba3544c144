#!/bin/bash
# The three reference tutorials, 10^4 iterations each, on the device (final build of the round)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 600 python -u -m pytest tests/test_tutorial_inference.py -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_tut.log 2>&1" \
 "timeout -k 10 600 python -u examples/fhn_gamma_inference.py --steps 10000 --out $O/tutorial_device.json > $O/tutorial_device.log 2>&1" \
 "timeout -k 10 600 python -u examples/fhn_gamma_inference.py --blocking --steps 10000 --out $O/tutorial_blocking_device.json > $O/tutorial_blocking_device.log 2>&1" \
 "timeout -k 10 600 python -u examples/fhn_gamma_inference.py --recordings 2 --steps 10000 --out $O/tutorial_ensemble_device.json > $O/tutorial_ensemble_device.log 2>&1"
