#!/bin/bash
# Lane-pair draw kernel: parity of the lane kernels, then C5/C3 A/B (pair on / off) on one box.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03d}
mkdir -p $O
A="--steps 30 --warmup 5 --no-cpu-baseline"
scripts/gpu_session.sh \
  "timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k 'lane_kernels or lane_pair or device_rng or full_size' > $O/pytest.log 2>&1" \
  "timeout -k 10 180 python bench.py --config c5 $A > $O/c5_pair.json 2> $O/c5_pair.err" \
  "DMT_LANE_PAIR=0 timeout -k 10 180 python bench.py --config c5 $A > $O/c5_single.json 2> $O/c5_single.err" \
  "DMT_LANE_PAIR=1 timeout -k 10 180 python bench.py --config c3 $A > $O/c3_pair.json 2> $O/c3_pair.err" \
  "DMT_LANE_PAIR=0 timeout -k 10 180 python bench.py --config c3 $A > $O/c3_single.json 2> $O/c3_single.err" \
  "timeout -k 10 180 python bench.py --config c5 $A > $O/c5_pair2.json 2> $O/c5_pair2.err"
