#!/bin/bash
# round 5: C5 on the packet layout's producer/consumer kernel (k_block_ps_pk, DMT_LANE_SPLIT=1)
# — its parity tests first, then kernel time per draw against the default packet kernel
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05j; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
S=("timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k 'split_packets or lane_kernels_bit_exact or c5' > $O/pytest.log 2>&1")
for r in 1 2; do
  S+=("timeout -k 10 150 python scripts/kbench.py --config c5 --mapping lane --accept --iters 20 > $O/c5_def_$r.json 2> $O/c5_def_$r.err")
  S+=("DMT_LANE_SPLIT=1 timeout -k 10 150 python scripts/kbench.py --config c5 --mapping lane --accept --iters 20 > $O/c5_split_$r.json 2> $O/c5_split_$r.err")
done
scripts/gpu_session.sh "${S[@]}"
for f in $O/c*.json; do echo "$f $(python -c "import json;print(round(json.load(open('$f'))['kernel_us'],1))")"; done
grep -E "passed|failed|PASS|FAIL" $O/pytest.log | tail -25
