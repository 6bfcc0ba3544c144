#!/bin/bash
# round 6, session H: which wave of C5's k_block_ps_pk sets the pace — timing probes that leave
# the results unchanged (DMT_PSPK_STUB=16: the producer draws every normal block twice; 32: the
# consumer runs every step's arithmetic twice) — and the hand-off through LDS counters instead of
# one barrier per chunk (DMT_PSPK_FLAGS=2, 3 slots), against the shipped kernel, interleaved,
# 2 rounds; GPU suite on flags3.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06h; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
V=$PWD/build_variants
S=("DMT_LIB_PATH=$V/libdmt_flags3.so timeout -k 10 300 python bench.py --config c5 --steps 4 --warmup 1 --calls-iters 0 --repeats 0 > $O/c5_flags3_check.json 2> $O/c5_flags3_check.err")
for r in 1 2; do
  S+=("timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 3 > $O/c5_full_$r.json 2> $O/c5_full_$r.err")
  for v in stub16 stub32 flags2 flags3; do
    S+=("DMT_LIB_PATH=$V/libdmt_$v.so timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 3 > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err")
  done
done
S+=("DMT_LIB_PATH=$V/libdmt_flags3.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_flags3.log 2>&1")
scripts/gpu_session.sh "${S[@]}"
tail -2 $O/pytest_flags3.log
for f in $O/c5_*.json; do python -c "import json;d=json.load(open('$f'));c=d.get('cpu_baseline') or {};print('$f', round(d['value']/1e10,4), round(d['roofline']['kernel_avg_us'],2), d.get('accept_rate'), c.get('decisions_identical'), c.get('decisions_total'))"; done
