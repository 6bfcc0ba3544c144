#!/bin/bash
# Round 2 final evidence on the final build: GPU suite, smoke, bench lines (C2 driver command,
# C2 200 iterations, C3, C5, each with its CPU leg), rocprofv3 kernel traces of the same commands.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zn
mkdir -p $O
NB="--no-cpu-baseline"
scripts/gpu_session.sh \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 $NB > $O/bench_c2_200.json 2> $O/bench_c2_200.err" \
 "timeout -k 10 400 python bench.py --config c3 --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err" \
 "timeout -k 10 400 python bench.py --config c5 --steps 20 --warmup 5 > $O/bench_c5.json 2> $O/bench_c5.err" \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 $NB > $O/prof_c2.log 2>&1" \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 --output-format csv -- python bench.py --config c3 --steps 20 --warmup 5 $NB > $O/prof_c3.log 2>&1" \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 --output-format csv -- python bench.py --config c5 --steps 20 --warmup 5 $NB > $O/prof_c5.log 2>&1"
