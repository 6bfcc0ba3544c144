#!/bin/bash
# Probe: a chunk's X°/W° rows stored as per-lane K-step packets (16-byte stores; timing only,
# build_variants/libdmt_pkt.so) against the default per-row stores. Draw-only (scripts/kbench.py),
# fixed selectors: uniform, or mixed by one accept of a random fraction (no acceptance dynamics).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03pkt}
mkdir -p $O
V=DMT_LIB_PATH=build_variants/libdmt_pkt.so
K="python scripts/kbench.py --mapping lane --iters 10"
scripts/gpu_session.sh \
  "timeout -k 10 150 $K --config c5 --mix 0.54 > $O/c5mix_def1.json" \
  "$V timeout -k 10 150 $K --config c5 --mix 0.54 > $O/c5mix_pkt1.json" \
  "timeout -k 10 150 $K --config c5 > $O/c5uni_def1.json" \
  "$V timeout -k 10 150 $K --config c5 > $O/c5uni_pkt1.json" \
  "timeout -k 10 150 $K --config c3 > $O/c3uni_def1.json" \
  "$V timeout -k 10 150 $K --config c3 > $O/c3uni_pkt1.json" \
  "timeout -k 10 150 $K --config c5 --mix 0.54 > $O/c5mix_def2.json" \
  "$V timeout -k 10 150 $K --config c5 --mix 0.54 > $O/c5mix_pkt2.json" \
  "timeout -k 10 150 $K --config c3 > $O/c3uni_def2.json" \
  "$V timeout -k 10 150 $K --config c3 > $O/c3uni_pkt2.json"
