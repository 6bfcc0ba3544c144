#!/bin/bash
# Round-2 baseline on HEAD: GPU suite, smoke, the driver's bench config, C3/C5 benches,
# rocprofv3 kernel trace of the driver's exact bench command.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02a
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2_driver.json 2> $O/bench_c2_driver.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2drv -o c2 --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_c2drv.log 2>&1" \
 "timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err" \
 "timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err"
