#!/bin/bash
# C2 kernel knobs at 200-iteration launches: consumer draw after the scan (late), producer
# Philox/Box-Muller scheduling groups 1 and 3 (default: no group barriers), base twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zq
mkdir -p $O
A="--gpus 1 --steps 200 --warmup 20 --no-cpu-baseline"
scripts/gpu_session.sh \
 "timeout -k 10 120 python bench.py $A > $O/base1.json 2> $O/base1.err" \
 "DMT_LIB_PATH=build_variants/libdmt_late.so timeout -k 10 120 python bench.py $A > $O/late1.json 2> $O/late1.err" \
 "DMT_LIB_PATH=build_variants/libdmt_g1.so timeout -k 10 120 python bench.py $A > $O/g1_1.json 2> $O/g1_1.err" \
 "DMT_LIB_PATH=build_variants/libdmt_g3.so timeout -k 10 120 python bench.py $A > $O/g3_1.json 2> $O/g3_1.err" \
 "timeout -k 10 120 python bench.py $A > $O/base2.json 2> $O/base2.err" \
 "DMT_LIB_PATH=build_variants/libdmt_late.so timeout -k 10 120 python bench.py $A > $O/late2.json 2> $O/late2.err" \
 "DMT_LIB_PATH=build_variants/libdmt_g1.so timeout -k 10 120 python bench.py $A > $O/g1_2.json 2> $O/g1_2.err" \
 "DMT_LIB_PATH=build_variants/libdmt_g3.so timeout -k 10 120 python bench.py $A > $O/g3_2.json 2> $O/g3_2.err"
