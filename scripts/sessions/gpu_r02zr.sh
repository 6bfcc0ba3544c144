#!/bin/bash
# Kogge–Stone lane fetches through DPP / permlane swaps (bit-identical to ds_bpermute):
# probe, OU parity tests, then A/B against the ds_bpermute build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zr
mkdir -p $O
A="--gpus 1 --steps 200 --warmup 20 --no-cpu-baseline"
D="--gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
V=build_variants/libdmt_base.so
scripts/gpu_session.sh \
 "timeout -k 10 60 scripts/probe_ksread > $O/probe.log 2>&1" \
 "timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py tests/test_multirank.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest.log 2>&1" \
 "timeout -k 10 120 python bench.py $A > $O/a_new1.json 2> $O/a_new1.err" \
 "DMT_LIB_PATH=$V timeout -k 10 120 python bench.py $A > $O/a_base1.json 2> $O/a_base1.err" \
 "timeout -k 10 120 python bench.py $A > $O/a_new2.json 2> $O/a_new2.err" \
 "DMT_LIB_PATH=$V timeout -k 10 120 python bench.py $A > $O/a_base2.json 2> $O/a_base2.err" \
 "timeout -k 10 120 python bench.py $D > $O/d_new.json 2> $O/d_new.err" \
 "DMT_LIB_PATH=$V timeout -k 10 120 python bench.py $D > $O/d_base.json 2> $O/d_base.err"
