#!/bin/bash
# Round-3 baseline on a fresh box: GPU suite, smoke, the driver's bench command, C3/C5 bench lines.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03a}
mkdir -p $O
scripts/gpu_session.sh \
  "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1" \
  "timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" \
  "timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2_driver.json 2> $O/bench_c2_driver.err" \
  "timeout -k 10 180 python bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err" \
  "timeout -k 10 180 python bench.py --config c5 --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err"
