#!/bin/bash
# round 6, session K: C5's producer requesting both 16-point pieces of each lane's 128-byte u.W
# line at once (DMT_PSPK_WLINE=1) against the shipped kernel (pieces requested 16 steps apart),
# interleaved, 2 rounds; PMC FETCH/WRITE of each; CPU-leg line and the GPU suite on the variant.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06k; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
V=$PWD/build_variants
B5="python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline --calls-iters 0 --repeats 0"
S=("DMT_LIB_PATH=$V/libdmt_wline.so timeout -k 10 300 python bench.py --config c5 --steps 4 --warmup 1 --calls-iters 0 --repeats 0 > $O/c5_wline_check.json 2> $O/c5_wline_check.err")
for r in 1 2; do
  S+=("timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 3 > $O/c5_full_$r.json 2> $O/c5_full_$r.err")
  S+=("DMT_LIB_PATH=$V/libdmt_wline.so timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 3 > $O/c5_wline_$r.json 2> $O/c5_wline_$r.err")
done
S+=("DMT_LIB_PATH=$V/libdmt_wline.so timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_wline_fetch -o f --output-format csv -- $B5 > $O/pmc_wline_fetch.log 2>&1"
    "DMT_LIB_PATH=$V/libdmt_wline.so timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_wline_write -o w --output-format csv -- $B5 > $O/pmc_wline_write.log 2>&1"
    "DMT_LIB_PATH=$V/libdmt_wline.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_wline.log 2>&1")
scripts/gpu_session.sh "${S[@]}"
tail -1 $O/pytest_wline.log
for f in $O/c5_*.json; do python -c "import json;d=json.load(open('$f'));c=d.get('cpu_baseline') or {};print('$f', round(d['value']/1e10,4), round(d['roofline']['kernel_avg_us'],2), d.get('accept_rate'), c.get('decisions_identical'), c.get('decisions_total'))"; done
python scripts/pmc_traffic.py --fetch $O/pmc_wline_fetch/f_counter_collection.csv --write $O/pmc_wline_write/w_counter_collection.csv --kernel "k_block_ps_pk<" --config c5 --skip 2 --tree $O/tree.txt --out $O/traffic_wline.json > /dev/null 2>&1
python -c "import json;d=json.load(open('$O/traffic_wline.json'));print('wline raw', d['fetch_bytes_per_unit']/1e9, d['write_bytes_per_unit']/1e9)"
