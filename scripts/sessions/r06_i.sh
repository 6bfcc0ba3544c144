#!/bin/bash
# round 6, session I: C5 with a helper wave per tile drawing the odd Philox blocks of every packet
# one packet ahead (DMT_PSPK_HELPER=1, three waves per workgroup) against the shipped two-wave
# kernel, interleaved, 2 rounds; a line with the CPU leg (decisions) and the GPU suite on it.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06i; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
V=$PWD/build_variants
S=("DMT_LIB_PATH=$V/libdmt_helper.so timeout -k 10 300 python bench.py --config c5 --steps 4 --warmup 1 --calls-iters 0 --repeats 0 > $O/c5_helper_check.json 2> $O/c5_helper_check.err")
for r in 1 2; do
  S+=("timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 3 > $O/c5_full_$r.json 2> $O/c5_full_$r.err")
  S+=("DMT_LIB_PATH=$V/libdmt_helper.so timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 3 > $O/c5_helper_$r.json 2> $O/c5_helper_$r.err")
done
S+=("DMT_LIB_PATH=$V/libdmt_helper.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_helper -o c5 --output-format csv -- python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 0 > $O/prof_helper.json 2> $O/prof_helper.log"
    "DMT_LIB_PATH=$V/libdmt_helper.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_helper.log 2>&1")
scripts/gpu_session.sh "${S[@]}"
tail -2 $O/pytest_helper.log
for f in $O/c5_*.json; do python -c "import json;d=json.load(open('$f'));c=d.get('cpu_baseline') or {};print('$f', round(d['value']/1e10,4), round(d['roofline']['kernel_avg_us'],2), d.get('accept_rate'), c.get('decisions_identical'), c.get('decisions_total'))"; done
python -c "
import csv,glob,statistics
f=glob.glob('$O/prof_helper/*kernel_trace.csv')[0]
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in csv.DictReader(open(f)) if 'k_block_ps_pk' in r['Kernel_Name']]
d=d[3:]
print('helper rocprof', len(d), round(statistics.median(d),2), round(statistics.mean(d),2))"
