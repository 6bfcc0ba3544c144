set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r01b
export TMPDIR=/tmp
O=gpurun_out/r01b
if [ "$1" != B ]; then
scripts/gpu_session.sh \
 "timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1" \
 "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1" \
 "timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err" \
 "timeout -k 10 400 python bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- python bench.py --steps 30 --no-cpu-baseline > $O/prof_c2.log 2>&1" \
 "timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c2_fetch -o f --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/pmc_c2_fetch.log 2>&1" \
 "timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c2_write -o w --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/pmc_c2_write.log 2>&1" \
 "timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_calib_fetch -o f --output-format csv -- scripts/calib_stream > $O/calib_f.log 2>&1" \
 "timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_calib_write -o w --output-format csv -- scripts/calib_stream > $O/calib_w.log 2>&1"
else
scripts/gpu_session.sh \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 --output-format csv -- python bench.py --config c3 --steps 20 --no-cpu-baseline > $O/prof_c3.log 2>&1" \
 "timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_c3_fetch -o f --output-format csv -- python bench.py --config c3 --steps 6 --warmup 2 --no-cpu-baseline > $O/pmc_c3_fetch.log 2>&1" \
 "timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_c3_write -o w --output-format csv -- python bench.py --config c3 --steps 6 --warmup 2 --no-cpu-baseline > $O/pmc_c3_write.log 2>&1"
fi
