#!/bin/bash
# round 5: k_block_ps_pk storing whole X° packets of a uniform wave as contiguous 1 KB rows
# through LDS (DMT_PSPK_XLDS=1, default) against the per-lane pieces (xl0); parity tests first
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05s; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
S=("timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k 'split_packets or lane_kernels_bit_exact or c5' > $O/pytest.log 2>&1")
for r in 1 2; do
  for v in def xl0; do
    if [ $v = def ]; then LP=$PWD/diffusionmcmctools.jl_amd/libdmt.so; else LP=$PWD/build_variants/libdmt_$v.so; fi
    S+=("DMT_LIB_PATH=$LP timeout -k 10 150 python scripts/kbench.py --config c5 --mapping lane --accept --iters 20 > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err")
  done
done
scripts/gpu_session.sh "${S[@]}"
grep -E "passed|failed" $O/pytest.log | tail -2
for f in $O/c*.json; do echo "$f $(python -c "import json;print(round(json.load(open('$f'))['kernel_us'],1))")"; done
