#!/bin/bash
# round 5: C5 packet-kernel A/B (HEAD base vs chunk-end piece stores + branch-free quadrants),
# GPU suite on the new tree, then the TD persistent-kernel probes (last: they may fault)
set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then LP=$PWD/build_variants/libdmt_base.so; else LP=$PWD/diffusionmcmctools.jl_amd/libdmt.so; fi
    DMT_LIB_PATH=$LP timeout -k 10 120 python -u scripts/kbench.py --config c5 --mapping lane --accept --iters 20 > $O/c5_${v}_$r.json 2>$O/c5_${v}_$r.err || exit 1
    echo "$v $r $(tail -c 400 $O/c5_${v}_$r.json)"
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc $?"; tail -3 $O/pytest.log
DMT_LIB_PATH=$PWD/build_variants/libdmt_tdni.so TD_DETAIL=2 timeout -k 10 150 python -u scripts/td_fault_probe.py > $O/td_tdni.log 2>&1 || { echo tdni failed; tail -3 $O/td_tdni.log; exit 2; }
tail -4 $O/td_tdni.log
DMT_LIB_PATH=$PWD/build_variants/libdmt_tdauxp.so TD_DETAIL=2 timeout -k 10 150 python -u scripts/td_fault_probe.py > $O/td_tdauxp.log 2>&1 || { echo tdauxp failed; tail -3 $O/td_tdauxp.log; exit 3; }
tail -4 $O/td_tdauxp.log
