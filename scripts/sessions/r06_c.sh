#!/bin/bash
# round 6, session C: the FHN step map on the default build — GPU suite
# and smoke (device == oracle bit for bit), the tutorial's kernels (k_block_wave), C3 (the FHN
# lane kernel) and C5 (32-point lane packets) bench lines with kernel traces.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06c; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
S=("timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1"
   "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1")
for r in 1 2; do
  S+=("timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tut_$r -o tut --output-format csv -- python examples/fhn_gamma_inference.py --steps 40 --burn-in 10 > $O/tut_$r.log 2>&1")
done
S+=("timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --calls-iters 0 --repeats 3 > $O/bench_c3.json 2> $O/bench_c3.err"
    "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 --output-format csv -- python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 0 > $O/prof_c3.json 2> $O/prof_c3.log"
    "timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --calls-iters 0 --repeats 3 > $O/bench_c5.json 2> $O/bench_c5.err"
    "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err")
scripts/gpu_session.sh "${S[@]}"
tail -2 $O/pytest.log; cat $O/smoke.log
for f in $O/bench_c*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];c=d.get('cpu_baseline') or {};print('$f', round(d['value']/1e10,4), round(r.get('kernel_avg_us',0),2), round(r['frac'],3), c.get('sample','')[:60], c.get('decisions_identical'), c.get('decisions_total'))"; done
for r in 1 2; do python -c "
import csv
rows=list(csv.DictReader(open('$O/tut_$r/tut_kernel_stats.csv')))
w=[r for r in rows if 'k_block_wave' in r['Name']]
tot=sum(float(r['TotalDurationNs']) for r in rows)/1e6/40
print('tut $r', [(r['Name'][22:45], round(float(r['AverageNs'])/1e3,1)) for r in w], 'all kernels ms/iter', round(tot,3))"; done
python -c "
import csv,glob,statistics
f=glob.glob('$O/prof_c3/*kernel_trace.csv')[0]
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in csv.DictReader(open(f)) if 'k_block<' in r['Kernel_Name']]
d=d[3:]
print('c3 k_block', len(d), round(statistics.median(d),2), round(statistics.mean(d),2))"
