#!/bin/bash
# round 5, shipped tree check: the GPU suite, smoke, and bench.py with no flags (the driver's defaults)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05t; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
scripts/gpu_session.sh \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1" \
 "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" \
 "timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err"
tail -1 $O/pytest.log; tail -1 $O/smoke.log
python -c "import json;d=json.load(open('$O/bench_default.json'));r=d['roofline'];print(d['value'], d['steps'], d['warmup'], r['frac'], r['kernel_avg_us'], r['kernel_avg_us_rocprof'], r['traffic_source'], r['rocprof_source'], r.get('stale_summaries'))"
