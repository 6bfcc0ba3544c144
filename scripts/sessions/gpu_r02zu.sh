#!/bin/bash
# Final build of the session (container re-created, tree rebuilt): GPU suite, smoke, the driver's
# bench command (with its CPU leg) and a rocprofv3 kernel trace of it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zu
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" \
 "timeout -k 10 300 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err" \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_c2.log 2>&1" \
 "timeout -k 10 400 python bench.py --config c5 --steps 20 --warmup 5 > $O/bench_c5.json 2> $O/bench_c5.err"
