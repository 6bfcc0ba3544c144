#!/bin/bash
# round 5: where k_block_ps_pk's consumer spends its time — timing stubs on C5 (wrong results):
# s2 no normals, s6 + no X° stores, s10 + no H/F loads (stores kept), s14 neither
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05m; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
S=()
for r in 1 2; do
  for v in s2 s6 s10 s14; do
    S+=("DMT_LIB_PATH=$PWD/build_variants/libdmt_$v.so DMT_LANE_SPLIT=1 timeout -k 10 150 python scripts/kbench.py --config c5 --mapping lane --accept --iters 20 > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err")
  done
done
scripts/gpu_session.sh "${S[@]}"
for f in $O/c*.json; do echo "$f $(python -c "import json;print(round(json.load(open('$f'))['kernel_us'],1))")"; done
