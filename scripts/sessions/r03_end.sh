#!/bin/bash
# Final tree of the round: GPU suite, smoke, the driver's bench command (with its CPU leg), the
# default bench, C3 and C5 bench lines, rocprofv3 kernel trace of the driver's command.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03end}
mkdir -p $O
scripts/gpu_session.sh \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1" \
 "timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2_driver.json 2> $O/bench_c2_driver.err" \
 "timeout -k 10 300 python bench.py > $O/bench_c2_default.json 2> $O/bench_c2_default.err" \
 "timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 > $O/bench_c3.json 2> $O/bench_c3.err" \
 "timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 > $O/bench_c5.json 2> $O/bench_c5.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_c2.json 2> $O/prof_c2.log"
