#!/bin/bash
# Shared-grid lane kernel (compile-time t/H strides, √dt table): same-box A/B against the
# previous build (build_variants/libdmt_old.so) on C5 and C3 draws, then the GPU suite, smoke,
# bench lines (C2 driver command, C3, C5 with CPU legs) and rocprofv3 traces of C3/C5.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02zt
mkdir -p $O
NB="--no-cpu-baseline"
OLD="DMT_LIB_PATH=$PWD/build_variants/libdmt_old.so"
K5="python scripts/kbench.py --config c5 --mapping lane --iters 20 --accept"
K3="python scripts/kbench.py --config c3 --mapping lane --iters 20 --accept"
scripts/gpu_session.sh \
 "timeout -k 10 180 $K5 > $O/c5_new_a.json 2> $O/c5_new_a.err" \
 "$OLD timeout -k 10 180 $K5 > $O/c5_old_a.json 2> $O/c5_old_a.err" \
 "timeout -k 10 180 $K5 > $O/c5_new_b.json 2> $O/c5_new_b.err" \
 "$OLD timeout -k 10 180 $K5 > $O/c5_old_b.json 2> $O/c5_old_b.err" \
 "timeout -k 10 180 $K3 > $O/c3_new_a.json 2> $O/c3_new_a.err" \
 "$OLD timeout -k 10 180 $K3 > $O/c3_old_a.json 2> $O/c3_old_a.err" \
 "timeout -k 10 180 $K3 > $O/c3_new_b.json 2> $O/c3_new_b.err" \
 "$OLD timeout -k 10 180 $K3 > $O/c3_old_b.json 2> $O/c3_old_b.err" \
 "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" \
 "timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err" \
 "timeout -k 10 400 python bench.py --config c3 --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err" \
 "timeout -k 10 400 python bench.py --config c5 --steps 20 --warmup 5 > $O/bench_c5.json 2> $O/bench_c5.err" \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 --output-format csv -- python bench.py --config c3 --steps 20 --warmup 5 $NB > $O/prof_c3.log 2>&1" \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o c5 --output-format csv -- python bench.py --config c5 --steps 20 --warmup 5 $NB > $O/prof_c5.log 2>&1"
