#!/bin/bash
# Round 4: (1) C5 packet kernels — register-staged packet stores (default) vs LDS-staged, lane
# pairs and single lanes; (2) C2 — the DPP scan tree (build_variants/libdmt_dpp.so) vs the
# ds_bpermute Kogge–Stone at the driver's command, interleaved, its parity against the oracle
# restated with the same tree, and device stamps of one launch; (3) the GPU suite.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04g}
mkdir -p $O
K="python scripts/kbench.py --mapping lane --config c5 --accept"
LV=build_variants/libdmt_lds.so
DV=build_variants/libdmt_dpp.so
BC="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --repeats 20 --calls-iters 0"
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread"
scripts/gpu_session.sh \
 "timeout -k 10 300 $PT tests/test_td_aux.py > $O/pytest_td.log 2>&1" \
 "timeout -k 10 150 $K > $O/c5_regpair1.json 2> $O/c5_regpair1.err" \
 "DMT_LANE_PAIR=0 timeout -k 10 150 $K > $O/c5_reg1.json 2> $O/c5_reg1.err" \
 "DMT_LIB_PATH=$LV timeout -k 10 150 $K > $O/c5_ldspair1.json 2> $O/c5_ldspair1.err" \
 "DMT_LIB_PATH=$LV DMT_LANE_PAIR=0 timeout -k 10 150 $K > $O/c5_lds1.json 2> $O/c5_lds1.err" \
 "timeout -k 10 150 $K > $O/c5_regpair2.json 2> $O/c5_regpair2.err" \
 "DMT_LANE_PAIR=0 timeout -k 10 150 $K > $O/c5_reg2.json 2> $O/c5_reg2.err" \
 "timeout -k 10 150 $BC > $O/c2_ks1.json 2> $O/c2_ks1.err" \
 "DMT_LIB_PATH=$DV timeout -k 10 150 $BC > $O/c2_dpp1.json 2> $O/c2_dpp1.err" \
 "timeout -k 10 150 $BC > $O/c2_ks2.json 2> $O/c2_ks2.err" \
 "DMT_LIB_PATH=$DV timeout -k 10 150 $BC > $O/c2_dpp2.json 2> $O/c2_dpp2.err" \
 "DMT_LIB_PATH=$DV DMT_ORACLE_LIB=build_variants/liboracle_dpp.so timeout -k 10 400 $PT tests/test_dropin.py tests/test_gpu_parity.py -k 'ou or c2 or c1 or headline or mcmc_run or resident or scan' > $O/pytest_dpp.log 2>&1" \
 "DMT_LIB_PATH=build_variants/libdmt_stamps.so timeout -k 10 120 python scripts/pc_stamps.py > $O/c2_stamps.jsonl 2> $O/c2_stamps.err" \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1"
