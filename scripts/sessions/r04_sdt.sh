#!/bin/bash
# Round 4: the packet kernel reading a shared grid's √dt from a per-point table (default) vs a
# square root per step (build_variants/libdmt_nosdt.so): lane/packet parity tests, C5 draw
# timing interleaved, the C5 bench line.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04q}
mkdir -p $O
K="python scripts/kbench.py --mapping lane --config c5 --accept"
NV=build_variants/libdmt_nosdt.so
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_path_buffers.py tests/test_td_aux.py -m gpu > $O/pytest_lane.log 2>&1 &&
timeout -k 10 150 $K > $O/c5_sdt1.json 2> $O/c5_sdt1.err &&
DMT_LIB_PATH=$NV timeout -k 10 150 $K > $O/c5_nosdt1.json 2> $O/c5_nosdt1.err &&
timeout -k 10 150 $K > $O/c5_sdt2.json 2> $O/c5_sdt2.err &&
DMT_LIB_PATH=$NV timeout -k 10 150 $K > $O/c5_nosdt2.json 2> $O/c5_nosdt2.err &&
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 > $O/bench_c5.json 2> $O/bench_c5.err
rc=$?
echo "session rc=$rc"
exit $rc
