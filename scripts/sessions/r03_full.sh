#!/bin/bash
# Full check after a change: GPU suite, smoke, the driver's bench command, the --api calls line
# (service on / off), and a rocprofv3 kernel trace of the driver's command.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03v}
mkdir -p $O
scripts/gpu_session.sh \
  "timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1" \
  "timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" \
  "timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2_driver.json 2> $O/bench_c2_driver.err" \
  "timeout -k 10 180 python bench.py --api calls --steps 500 --warmup 20 --no-cpu-baseline --repeats 0 > $O/bench_c2_calls.json 2> $O/bench_c2_calls.err" \
  "DMT_SERVICE=0 timeout -k 10 180 python bench.py --api calls --steps 500 --warmup 20 --no-cpu-baseline --repeats 0 > $O/bench_c2_calls_nosvc.json 2> $O/bench_c2_calls_nosvc.err" \
  "timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o c2 --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2_prof.json 2> $O/bench_c2_prof.err"
