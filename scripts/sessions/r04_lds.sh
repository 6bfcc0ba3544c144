#!/bin/bash
# Round 4: C5 packet kernels — lane pairs (default for C5) vs one lane per recording (LDS-staged
# packet stores) vs the register-staged previous build; time-dependent ã(t) GPU tests; the
# whole GPU suite.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04e}
mkdir -p $O
K="python scripts/kbench.py --mapping lane --config c5 --accept"
RS=build_variants/libdmt_regstage.so
scripts/gpu_session.sh \
 "timeout -k 10 150 $K > $O/c5_pair1.json 2> $O/c5_pair1.err" \
 "DMT_LANE_PAIR=0 timeout -k 10 150 $K > $O/c5_lds1.json 2> $O/c5_lds1.err" \
 "DMT_LIB_PATH=$RS timeout -k 10 150 $K > $O/c5_reg1.json 2> $O/c5_reg1.err" \
 "timeout -k 10 150 $K > $O/c5_pair2.json 2> $O/c5_pair2.err" \
 "DMT_LANE_PAIR=0 timeout -k 10 150 $K > $O/c5_lds2.json 2> $O/c5_lds2.err" \
 "DMT_LIB_PATH=$RS timeout -k 10 150 $K > $O/c5_reg2.json 2> $O/c5_reg2.err" \
 "timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_td_aux.py > $O/pytest_td.log 2>&1" \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1"
