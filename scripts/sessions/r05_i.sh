#!/bin/bash
# round 5: C5 packet kernel with 8-step guiding-term chunks (pk8, DMT_PK_KCHUNK=8) against the
# default 4; C3 with the lane kernel's automatic two-chunk prefetch (default) against one (a1);
# then the GPU suite on the default build
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05i; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
DEF=$PWD/diffusionmcmctools.jl_amd/libdmt.so
S=()
for r in 1 2; do
  S+=("DMT_LIB_PATH=$DEF timeout -k 10 150 python scripts/kbench.py --config c5 --mapping lane --accept --iters 20 > $O/c5_def_$r.json 2> $O/c5_def_$r.err")
  S+=("DMT_LIB_PATH=$PWD/build_variants/libdmt_pk8.so timeout -k 10 150 python scripts/kbench.py --config c5 --mapping lane --accept --iters 20 > $O/c5_pk8_$r.json 2> $O/c5_pk8_$r.err")
  S+=("DMT_LIB_PATH=$DEF timeout -k 10 150 python scripts/kbench.py --config c3 --mapping lane --accept --iters 20 > $O/c3_def_$r.json 2> $O/c3_def_$r.err")
  S+=("DMT_LIB_PATH=$PWD/build_variants/libdmt_a1.so timeout -k 10 150 python scripts/kbench.py --config c3 --mapping lane --accept --iters 20 > $O/c3_a1_$r.json 2> $O/c3_a1_$r.err")
done
S+=("timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1")
scripts/gpu_session.sh "${S[@]}"
for f in $O/c*.json; do echo "$f $(python -c "import json;print(round(json.load(open('$f'))['kernel_us'],1))")"; done
tail -3 $O/pytest.log
