#!/bin/bash
# round 5: tutorial A/B (r04 base vs the FHN drift reassociation: the serial recursion's chain
# 8 -> 5 dependent fp64 operations), C5 A/B (fp32 Box-Muller log + quadrants), GPU suite, the
# driver's C2 command twice, the C5 line
set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
lib() { if [ $1 = base ]; then echo $PWD/build_variants/libdmt_base.so; else echo $PWD/diffusionmcmctools.jl_amd/libdmt.so; fi; }
for r in 1 2; do
  for v in base new; do
    DMT_LIB_PATH=$(lib $v) timeout -k 10 200 python -u examples/fhn_gamma_inference.py --steps 1000 --burn-in 100 > $O/tut_${v}_$r.log 2>&1 || { echo tut failed; tail -3 $O/tut_${v}_$r.log; exit 1; }
    echo "tut $v $r $(tail -1 $O/tut_${v}_$r.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['run_seconds']/d['steps']*1e3,3),'ms/iter')")"
  done
done
for r in 1 2; do
  for v in base new; do
    DMT_LIB_PATH=$(lib $v) timeout -k 10 120 python -u scripts/kbench.py --config c5 --mapping lane --accept --iters 20 > $O/c5_${v}_$r.json 2>$O/c5_${v}_$r.err || exit 2
    echo "c5 $v $r $(python -c "import json;d=json.load(open('$O/c5_${v}_$r.json'));print(round(d['kernel_us'],1))")"
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc $?"; tail -3 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c2_$r.json 2>$O/bench_c2_$r.err || { echo bench failed; tail -5 $O/bench_c2_$r.err; exit 4; }
  python -c "import json;d=json.load(open('$O/bench_c2_$r.json'));print('c2', d['value'], d['roofline']['kernel_avg_us'], d['repeats']['value_median'], d['decisions_identical'], d['decisions_total'], d['separate_calls']['us_per_iteration_c'])"
done
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 3 --calls-iters 0 > $O/bench_c5.json 2>$O/bench_c5.err || { echo c5 bench failed; tail -5 $O/bench_c5.err; exit 5; }
python -c "import json;d=json.load(open('$O/bench_c5.json'));print('c5', d['value'], d['roofline']['kernel_avg_us'], d['roofline']['frac'], d['decisions_identical'], d['decisions_total'])"
