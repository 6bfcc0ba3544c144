#!/bin/bash
# Round 4: C5 packet kernels — register-staged packet stores (default) vs LDS-staged
# (build_variants/libdmt_lds.so), each with lane pairs (default for C5) and one lane per
# recording; the time-dependent aux tests (OU now too) and the whole GPU suite on the default build.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04f}
mkdir -p $O
K="python scripts/kbench.py --mapping lane --config c5 --accept"
LV=build_variants/libdmt_lds.so
scripts/gpu_session.sh \
 "timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_td_aux.py > $O/pytest_td.log 2>&1" \
 "timeout -k 10 150 $K > $O/c5_regpair1.json 2> $O/c5_regpair1.err" \
 "DMT_LANE_PAIR=0 timeout -k 10 150 $K > $O/c5_reg1.json 2> $O/c5_reg1.err" \
 "DMT_LIB_PATH=$LV timeout -k 10 150 $K > $O/c5_ldspair1.json 2> $O/c5_ldspair1.err" \
 "DMT_LIB_PATH=$LV DMT_LANE_PAIR=0 timeout -k 10 150 $K > $O/c5_lds1.json 2> $O/c5_lds1.err" \
 "timeout -k 10 150 $K > $O/c5_regpair2.json 2> $O/c5_regpair2.err" \
 "DMT_LANE_PAIR=0 timeout -k 10 150 $K > $O/c5_reg2.json 2> $O/c5_reg2.err" \
 "DMT_LIB_PATH=build_variants/libdmt_stamps.so timeout -k 10 120 python scripts/pc_stamps.py > $O/c2_stamps.jsonl 2> $O/c2_stamps.err" \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1"
