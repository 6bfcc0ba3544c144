#!/bin/bash
# round 5: k_block_ps_pk's consumer with its H, F chunks 3 ahead (ring of 4, default) against 1
# ahead (r2), and the consumer alone with the ring (r4stc); parity tests of the split kernels
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05l; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
S=("timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k 'split_packets or lane_kernels_bit_exact' > $O/pytest.log 2>&1")
for r in 1 2; do
  for v in def r2 r4stc; do
    if [ $v = def ]; then LP=$PWD/diffusionmcmctools.jl_amd/libdmt.so; else LP=$PWD/build_variants/libdmt_$v.so; fi
    S+=("DMT_LIB_PATH=$LP DMT_LANE_SPLIT=1 timeout -k 10 150 python scripts/kbench.py --config c5 --mapping lane --accept --iters 20 > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err")
  done
done
scripts/gpu_session.sh "${S[@]}"
for f in $O/c*.json; do echo "$f $(python -c "import json;print(round(json.load(open('$f'))['kernel_us'],1))")"; done
grep -E "passed|failed|PASS|FAIL|Error" $O/pytest.log | tail -12
