#!/bin/bash
# round 6, session L: C2's resident kernel with the decision posted before the consumer's X°
# stores and the next proposal formed in the producer's registers before B2 (DMT_PC_EARLY=1)
# against the same source without it (base: the decision computed before the stores) and the
# final tree f9629866 (f962), and early with the consumer's own steps proposed before B2 (earlyc), interleaved, 3 rounds; CPU-leg line and GPU suite on early.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06l; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
V=$PWD/build_variants
S=("DMT_LIB_PATH=$V/libdmt_early.so timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --repeats 0 --calls-iters 0 > $O/c2_early_check.json 2> $O/c2_early_check.err")
for r in 1 2 3; do
  for v in f962 base early earlyc; do
    S+=("DMT_LIB_PATH=$V/libdmt_$v.so timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --repeats 9 --calls-iters 0 > $O/c2_${v}_$r.json 2> $O/c2_${v}_$r.err")
  done
done
S+=("DMT_LIB_PATH=$V/libdmt_early.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_early.log 2>&1")
scripts/gpu_session.sh "${S[@]}"
tail -1 $O/pytest_early.log
for f in $O/c2_*.json; do python -c "import json;d=json.load(open('$f'));c=d.get('cpu_baseline') or {};print('$f', round(d['value']/1e10,4), round(d['roofline']['kernel_avg_us'],2), round(d['repeats']['value_median']/1e10,4) if d.get('repeats') else None, c.get('decisions_identical'), c.get('decisions_total'))"; done
