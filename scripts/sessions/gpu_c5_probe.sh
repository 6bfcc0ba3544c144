cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r01k
mkdir -p $O
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
scripts/gpu_session.sh \
 "timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 20 --warmup 3 > $O/c5_lane.json 2> $O/c5_lane.err" \
 "timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --steps 5 --warmup 1 --mapping wave > $O/c5_wave.json 2> $O/c5_wave.err" \
 "timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 5 --warmup 1 --mapping wave > $O/c3_wave.json 2> $O/c3_wave.err" \
 "timeout -s KILL 150 rocprofv3 --pmc $P1 -d $O/c5_p1 -o p --output-format csv -- python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > $O/c5_p1.log 2>&1"
