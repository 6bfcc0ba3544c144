#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r01q
mkdir -p $O
steps=()
for k in 4 8 16; do
  if [ $k = 4 ]; then LIB=""; else LIB="DMT_LIB_PATH=$PWD/dbgv/libdmt_k$k.so"; fi
  steps+=("$LIB timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 10 --warmup 3 > $O/c3_k$k.json 2> $O/c3_k$k.err")
  steps+=("$LIB timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 10 --warmup 3 > $O/c5_k$k.json 2> $O/c5_k$k.err")
done
steps+=("DMT_LIB_PATH=$PWD/dbgv/libdmt_k16.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_k16.log 2>&1")
scripts/gpu_session.sh "${steps[@]}"
