#!/bin/bash
# round 5: the resident MCMC service with the gate's host words read ahead (DMT_SVC_PEEK=1,
# default) against the plain gate (nopeek): the caller's separate-call loop per C2 iteration
# (bench.py separate_calls, 1 000 iterations from C); peek2: read after the scan; the service and deferred-call tests first
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05p}; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
S=("timeout -k 10 600 python -u -m pytest tests/test_deferred.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k 'deferred or service or svc or mcmc_run or separate' > $O/pytest.log 2>&1")
for r in 1 2; do
  for v in def peek2 nopeek; do
    if [ $v = def ]; then LP=$PWD/diffusionmcmctools.jl_amd/libdmt.so; else LP=$PWD/build_variants/libdmt_$v.so; fi
    S+=("DMT_LIB_PATH=$LP timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --calls-iters 1000 --repeats 3 > $O/c2_${v}_$r.json 2> $O/c2_${v}_$r.err")
  done
done
scripts/gpu_session.sh "${S[@]}"
tail -2 $O/pytest.log
for f in $O/c2_*.json; do python -c "import json;d=json.load(open('$f'));s=d['separate_calls'];print('$f', round(d['value']/1e10,3), round(s['us_per_iteration_c'],2), round(s['us_per_iteration_python_ctypes'],2))"; done
