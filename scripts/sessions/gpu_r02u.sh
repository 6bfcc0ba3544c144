#!/bin/bash
# Round 2: one vs two producer waves per block (k_mcmc_resident_pc<NP>), C2 200 iterations, + parity.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02u
mkdir -p $O
A="--gpus 1 --steps 200 --warmup 20 --no-cpu-baseline"
scripts/gpu_session.sh \
 "DMT_MCMC_PC=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k 'producer_consumer or persistent_paths' > $O/pytest_np2.log 2>&1" \
 "timeout -k 10 120 python bench.py $A > $O/np1.json 2> $O/np1.err" \
 "DMT_MCMC_PC=2 timeout -k 10 120 python bench.py $A > $O/np2.json 2> $O/np2.err" \
 "DMT_MCMC_PC=2 DMT_LIB_PATH=build_variants/libdmt_stubp2.so timeout -k 10 120 python bench.py $A > $O/stubp2.json 2> $O/stubp2.err" \
 "DMT_MCMC_PC=2 DMT_LIB_PATH=build_variants/libdmt_stubc2.so timeout -k 10 120 python bench.py $A > $O/stubc2.json 2> $O/stubc2.err"
