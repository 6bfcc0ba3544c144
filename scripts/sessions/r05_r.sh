#!/bin/bash
# round 5: C3 lane kernel with a ring of 4 register sets (3 chunks of 4 steps ahead; spills 60
# bytes) and the generic ring of 3 (= the default's two ahead) against the default
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05r; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
S=()
for r in 1 2; do
  for v in def ring3 ring4; do
    if [ $v = def ]; then LP=$PWD/diffusionmcmctools.jl_amd/libdmt.so; else LP=$PWD/build_variants/libdmt_$v.so; fi
    S+=("DMT_LIB_PATH=$LP timeout -k 10 150 python scripts/kbench.py --config c3 --mapping lane --accept --iters 20 > $O/c3_${v}_$r.json 2> $O/c3_${v}_$r.err")
  done
done
scripts/gpu_session.sh "${S[@]}"
for f in $O/c*.json; do echo "$f $(python -c "import json;print(round(json.load(open('$f'))['kernel_us'],1))")"; done
