#!/bin/bash
# round 5: where the driver's single timed C2 call spends its time beyond the kernel — libdmt's
# host-side phases per dmt_mcmc_run (DMT_HOST_PROFILE) at the driver's command, and the same
# command with 20 warm-up calls
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05u; mkdir -p $O
python scripts/provenance.py > $O/tree.txt
scripts/gpu_session.sh \
 "DMT_HOST_PROFILE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --calls-iters 0 --repeats 5 > $O/c2_w5.json 2> $O/c2_w5.err" \
 "DMT_HOST_PROFILE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 20 --no-cpu-baseline --calls-iters 0 --repeats 5 > $O/c2_w20.json 2> $O/c2_w20.err"
for w in w5 w20; do python -c "import json;d=json.load(open('$O/c2_$w.json'));print('$w', round(d['value']/1e10,3), round(d['ms_per_step']*20e3,1), round(d['repeats']['ms_per_step_median']*20e3,1))"; grep -v "^$" $O/c2_$w.err | tail -12; done
