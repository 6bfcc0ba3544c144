#!/bin/bash
# round 6, session J: C5 with the consumer drawing a share of the producer's normal blocks one
# packet ahead (DMT_PSPK_CSHARE=3: every third block, 4: every fourth) against the shipped
# kernel, interleaved, 2 rounds; CPU-leg lines (decisions) and the GPU suite on both variants.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06j; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
V=$PWD/build_variants
S=()
for v in cshare3 cshare4; do
  S+=("DMT_LIB_PATH=$V/libdmt_$v.so timeout -k 10 300 python bench.py --config c5 --steps 4 --warmup 1 --calls-iters 0 --repeats 0 > $O/c5_${v}_check.json 2> $O/c5_${v}_check.err")
done
for r in 1 2; do
  S+=("timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 3 > $O/c5_full_$r.json 2> $O/c5_full_$r.err")
  for v in cshare3 cshare4; do
    S+=("DMT_LIB_PATH=$V/libdmt_$v.so timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 3 > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err")
  done
done
for v in cshare3 cshare4; do
  S+=("DMT_LIB_PATH=$V/libdmt_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1")
done
scripts/gpu_session.sh "${S[@]}"
tail -1 $O/pytest_cshare3.log $O/pytest_cshare4.log
for f in $O/c5_*.json; do python -c "import json;d=json.load(open('$f'));c=d.get('cpu_baseline') or {};print('$f', round(d['value']/1e10,4), round(d['roofline']['kernel_avg_us'],2), d.get('accept_rate'), c.get('decisions_identical'), c.get('decisions_total'))"; done
