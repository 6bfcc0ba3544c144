#!/bin/bash
# round 5: C3 lane kernel (k_block, fp64 FHN) prefetch depth — one chunk of 4 steps ahead (base),
# two chunks of 4 (a2, DMT_LANE_AHEAD=2), one chunk of 8 (k8), two chunks of 8 (a2k8): kernel
# time per draw (device events, draw + accept loop), interleaved twice; then the C2 line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
S=()
for r in 1 2; do
  for v in base a2 k8 a2k8; do
    S+=("DMT_LIB_PATH=$PWD/build_variants/libdmt_$v.so timeout -k 10 150 python scripts/kbench.py --config c3 --mapping lane --accept --iters 20 > $O/c3_${v}_$r.json 2> $O/c3_${v}_$r.err")
  done
done
S+=("timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err")
scripts/gpu_session.sh "${S[@]}"
for f in $O/c3_*.json; do echo "$f $(python -c "import json;print(round(json.load(open('$f'))['kernel_us'],1))")"; done
