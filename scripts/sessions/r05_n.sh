#!/bin/bash
# round 5: is k_block_ps_pk's consumer bound by its H, F load instructions?  Timing stub 16 loads
# the same H, F bytes with 16-byte loads (4x fewer instructions; wrong lanes, wrong results);
# s18 = the same without the producer's normals (compare r05m s2: 1 243-1 245 µs)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05n; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
S=()
for r in 1 2; do
  for v in def s16 s18; do
    if [ $v = def ]; then LP=$PWD/diffusionmcmctools.jl_amd/libdmt.so; else LP=$PWD/build_variants/libdmt_$v.so; fi
    S+=("DMT_LIB_PATH=$LP timeout -k 10 150 python scripts/kbench.py --config c5 --mapping lane --accept --iters 20 > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err")
  done
done
scripts/gpu_session.sh "${S[@]}"
for f in $O/c*.json; do echo "$f $(python -c "import json;print(round(json.load(open('$f'))['kernel_us'],1))")"; done
