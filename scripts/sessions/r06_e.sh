#!/bin/bash
# round 6, session E: C5 — the split packet kernel's consumer reading its H, F chunks through an
# LDS-DMA ring (global_load_lds_dwordx4, DMT_PSPK_GLDS=1; 3 or 4 chunks in flight: glds4, glds5)
# against the register ring (nopair: DMT_PSPK_PAIR=0; pair: the whole-line stores), GPU suite on
# glds4, interleaved timing, PMC FETCH/WRITE and a kernel trace of each.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06e; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
V=$PWD/build_variants
VS="glds4 glds5 nopair pair"
S=("DMT_LIB_PATH=$V/libdmt_glds4.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_glds4.log 2>&1")
for r in 1 2; do
  for v in $VS; do
    S+=("DMT_LIB_PATH=$V/libdmt_$v.so timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 3 > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err")
  done
done
B5="python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline --calls-iters 0 --repeats 0"
for v in $VS; do
  S+=("DMT_LIB_PATH=$V/libdmt_$v.so timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_${v}_fetch -o f --output-format csv -- $B5 > $O/pmc_${v}_fetch.log 2>&1")
  S+=("DMT_LIB_PATH=$V/libdmt_$v.so timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_${v}_write -o w --output-format csv -- $B5 > $O/pmc_${v}_write.log 2>&1")
  S+=("DMT_LIB_PATH=$V/libdmt_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o c5 --output-format csv -- python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 0 > $O/prof_$v.json 2> $O/prof_$v.log")
done
scripts/gpu_session.sh "${S[@]}"
tail -2 $O/pytest_glds4.log
for f in $O/c5_*.json; do python -c "import json;d=json.load(open('$f'));print('$f', round(d['value']/1e10,4), round(d['roofline']['kernel_avg_us'],2))"; done
for v in $VS; do
  python scripts/pmc_traffic.py --fetch $O/pmc_${v}_fetch/f_counter_collection.csv --write $O/pmc_${v}_write/w_counter_collection.csv --kernel "k_block_ps_pk<" --config c5 --skip 2 --tree $O/tree.txt --out $O/traffic_$v.json > /dev/null 2>&1
  python -c "import json;d=json.load(open('$O/traffic_$v.json'));print('$v', {k: v for k, v in d.items() if 'bytes' in k})"
  python -c "
import csv,glob,statistics
f=glob.glob('$O/prof_$v/*kernel_trace.csv')[0]
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3 for r in csv.DictReader(open(f)) if 'k_block_ps_pk' in r['Kernel_Name']]
d=d[3:]
print('$v', len(d), round(statistics.median(d),2), round(min(d),2))"
done
