#!/bin/bash
# Round 4: per-iteration device stamps of one C2 workgroup (where a k_mcmc_resident_pc
# iteration's time goes: consumer chain, producer draw, the two barriers' waits).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04k}
mkdir -p $O
DMT_LIB_PATH=build_variants/libdmt_stamps.so timeout -k 10 120 python scripts/pc_stamps.py > $O/c2_stamps.jsonl 2> $O/c2_stamps.err
