#!/bin/bash
# GPU suite, tutorial profiles (plain + blocking), C3-scale aux kernels (chunked filter), C2 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_tut -o tut --output-format csv -- python examples/fhn_gamma_inference.py --steps 300 --burn-in 100 > $O/prof_tut.log 2>&1" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_tutb -o tutb --output-format csv -- python examples/fhn_gamma_inference.py --blocking --steps 200 --burn-in 50 > $O/prof_tutb.log 2>&1" \
 "timeout -k 10 300 python scripts/bench_aux.py > $O/aux_c3.jsonl 2> $O/aux_c3.err" \
 "timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err"
