#!/bin/bash
# round 6, session F: C3's memory pattern without its arithmetic (scripts/c3_mem_probe: 1-6 chunks
# of 4 steps loaded ahead, and a flat stream of the same bytes), C3 split into producer/consumer
# waves (DMT_LANE_SPLIT=1, k_block_ps) against the single wave, interleaved; C5 on the shipped
# PAIR default.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06f; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
S=("timeout -k 10 120 scripts/c3_mem_probe > $O/probe1.jsonl 2> $O/probe1.err")
for r in 1 2; do
  S+=("timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 3 > $O/c3_single_$r.json 2> $O/c3_single_$r.err")
  S+=("DMT_LANE_SPLIT=1 timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --calls-iters 0 --repeats 3 > $O/c3_split_$r.json 2> $O/c3_split_$r.err")
done
S+=("timeout -k 10 120 scripts/c3_mem_probe > $O/probe2.jsonl 2> $O/probe2.err"
    "timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --calls-iters 0 --repeats 3 > $O/c5_pair.json 2> $O/c5_pair.err")
scripts/gpu_session.sh "${S[@]}"
cat $O/probe1.jsonl $O/probe2.jsonl
for f in $O/c*.json; do python -c "import json;d=json.load(open('$f'));r=d['roofline'];c=d.get('cpu_baseline') or {};print('$f', round(d['value']/1e10,4), round(r['kernel_avg_us'],2), r['kernel'], c.get('decisions_identical'), c.get('decisions_total'))"; done
