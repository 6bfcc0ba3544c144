#!/bin/bash
# round 6, session M: the shipped tree's bench lines as the driver runs them, now quoting the
# round-6 summaries of the same tree (digest f9629866af0af08f): no flags, the 20-iteration
# command, C5 and C3; smoke().
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06m; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
scripts/gpu_session.sh \
 "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" \
 "timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2_driver.json 2> $O/bench_c2_driver.err" \
 "timeout -k 10 300 python bench.py --config c5 > $O/bench_c5.json 2> $O/bench_c5.err" \
 "timeout -k 10 300 python bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err"
cat $O/smoke.log
for f in $O/bench_*.json; do python -c "
import json;d=json.load(open('$f'));r=d['roofline'];c=d.get('cpu_baseline') or {}
print('$f', round(d['value']/1e10,4), round(r['kernel_avg_us'],2), round(r['frac'],3), r.get('kernel_avg_us_rocprof'), r.get('traffic'), r.get('rocprof_source'), r.get('traffic_source'), (r.get('issue') or {}).get('source') if isinstance(r.get('issue'), dict) else r.get('issue'), r.get('stale_summaries'), c.get('decisions_identical'), c.get('decisions_total'))"; done
