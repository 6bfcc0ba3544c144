#!/bin/bash
# Profiles the C2 bench (rocprofv3): kernel trace + stats, then separate FETCH_SIZE and
# WRITE_SIZE passes and the calibration program (scripts/calib_stream).  Output: $1 (dir).
set -o pipefail
O=${1:-gpurun_out/prof}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o c2 --output-format csv -- python bench.py --steps 50 --no-cpu-baseline > $O/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o f --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o w --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/write.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $O/calib_fetch -o f --output-format csv -- scripts/calib_stream > $O/calib_f.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $O/calib_write -o w --output-format csv -- scripts/calib_stream > $O/calib_w.log 2>&1 || exit $?
