#!/bin/bash
# Round 4, first call: GPU suite on the round-3 tree; the C5 layout probe (timing, then separate
# FETCH_SIZE / WRITE_SIZE passes); the real C5 draw inside a draw + accept loop for reference.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04a}
mkdir -p $O
K="python scripts/kbench.py"
P=scripts/c5_layout_probe
scripts/gpu_session.sh \
 "timeout -k 10 60 $P 512 10 > $O/probe.jsonl 2> $O/probe.err" \
 "timeout -k 10 150 $K --config c5 --mapping lane --accept > $O/c5_real.json 2> $O/c5_real.err" \
 "timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o f --output-format csv -- $P 512 3 > $O/pmc_fetch.log 2>&1" \
 "timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o w --output-format csv -- $P 512 3 > $O/pmc_write.log 2>&1" \
 "timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1"
