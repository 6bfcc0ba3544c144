#!/bin/bash
# round 6, session G: where C5's draw goes on the shipped k_block_ps_pk (whole-line stores):
# timing stubs (DMT_PSPK_STUB, wrong results, timing only) — 1: producer alone (no recursion),
# 2: consumer alone (no normals), 3: neither (the memory traffic and the hand-off), 12: no H, F
# loads and no X° stores — against the full kernel, interleaved, two rounds.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
V=$PWD/build_variants
S=()
for r in 1 2; do
  S+=("timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 3 > $O/c5_full_$r.json 2> $O/c5_full_$r.err")
  for v in stub1 stub2 stub3 stub12; do
    S+=("DMT_LIB_PATH=$V/libdmt_$v.so timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 3 > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err")
  done
done
scripts/gpu_session.sh "${S[@]}"
for f in $O/c5_*.json; do python -c "import json;d=json.load(open('$f'));print('$f', round(d['value']/1e10,4), round(d['roofline']['kernel_avg_us'],2))"; done
