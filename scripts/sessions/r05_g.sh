#!/bin/bash
# round 5: the tutorial's serial FHN recursion (k_block_wave, wave S) with its LDS rows 1, 4
# (default) and 8 steps ahead: rocprofv3 kernel stats of 300 tutorial iterations each; tutorial
# parity tests on the default
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05g; mkdir -p $O
for v in sp1 new sp8; do
  if [ $v = new ]; then LP=$PWD/diffusionmcmctools.jl_amd/libdmt.so; else LP=$PWD/build_variants/libdmt_$v.so; fi
  DMT_LIB_PATH=$LP timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o tut --output-format csv -- python examples/fhn_gamma_inference.py --steps 300 --burn-in 100 > $O/tut_$v.log 2>&1 || { echo "$v failed"; tail -3 $O/tut_$v.log; exit 1; }
  python - <<PY
import csv
rows=list(csv.DictReader(open("$O/prof_$v/tut_kernel_stats.csv")))
tot=sum(float(r['TotalDurationNs']) for r in rows)
w=[r for r in rows if 'k_block_wave' in r['Name']]
print("$v", "k_block_wave avg us", [round(float(r['AverageNs'])/1e3,1) for r in w], "kernel ms/iter", round(tot/1e6/300,3))
PY
done
timeout -k 10 600 python -u -m pytest tests/test_tutorial_inference.py tests/test_reference_tutorials.py tests/test_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc $?"; tail -2 $O/pytest.log
